# PMC comparison of library variants (one counter group per rocprofv3 pass).
# usage: VARIANTS="il" CFG=c2 ARGS="--mode separate" bash tools/gpu/pmc_ab.sh
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/pmc_ab; mkdir -p $O
CFG=${CFG:-c2}; VARIANTS=${VARIANTS:-il}; ARGS=${ARGS:---mode separate}
cd /tmp && export TMPDIR=/tmp
for v in cur $VARIANTS; do
  if [ $v = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$v.so; fi
  n=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum"; do
    n=$((n+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d $O/$v/p$n -o run --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 10 --warmup 2 $ARGS > $O/$v.p$n.log 2>&1 || { echo "pmc $v $grp failed"; tail -5 $O/$v.p$n.log; }
  done
  python3 $R/tools/pmc_report.py $O/$v $CFG $O/traffic_$v.json > /dev/null
  python3 - $O/traffic_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, e in d["kernels"].items():
    if "chachapoly" not in k and "gcm" not in k: continue
    w = e.get("SQ_WAVES", 1) or 1
    print(sys.argv[2], k, {x: round(y / w, 1) if x.startswith("SQ_") and x != "SQ_WAVES" else round(y) for x, y in e.items()})
PY
done

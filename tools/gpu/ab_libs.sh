# A/B of library variants on one box: the current lib vs noise-c_amd/ab/libnoise_aead_hip_$VARIANTS.so,
# interleaved rounds.  usage: VARIANTS="il" CFGS="c2" ARGS="--mode separate" bash tools/gpu/ab_libs.sh
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/ab_libs; mkdir -p $O
CFGS=${CFGS:-c2}; VARIANTS=${VARIANTS:-il}; ARGS=${ARGS:-}; ROUNDS=${ROUNDS:-2}
for i in $(seq $ROUNDS); do
  for v in cur $VARIANTS; do
    if [ $v = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$v.so; fi
    for c in $CFGS; do
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 8 $ARGS > $O/$v.$c.$i.json 2> $O/$v.$c.$i.err || { tail -20 $O/$v.$c.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$v.$c.$i.json'));print('$v $c',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],'seal',d['seal_gibs'],'open',d['open_gibs'])"
    done
  done
done

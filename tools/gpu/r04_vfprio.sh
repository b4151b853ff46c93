# Round 4: verify-first C2 with the AUTH pass at top priority (default) vs
# without (variant library NA_SOLO_NO_AUTH_PRIO), interleaved bench lines.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_vfprio}; mkdir -p $O
for rep in 1 2 3; do
  for v in prio noprio; do
    L=""; [ $v = noprio ] && L=$R/noise-c_amd/ab/libnoise_aead_hip_noprio.so
    NOISE_AEAD_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --verify-first > $O/c2_${v}_$rep.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${v}_$rep.json'));print('$v $rep',d['value'],d['roofline']['avg_launch_ms'],d['open_gibs'],d.get('verified'))"
  done
done

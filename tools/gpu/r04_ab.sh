# Round 4: interleaved A/B of the library against a variant build
# (noise-c_amd/ab/libnoise_aead_hip_$VAR.so) over bench configs.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_ab}; mkdir -p $O
VAR=${VAR:-base}
for rep in 1 2 3; do
  for c in ${CFGS:-c2 c4 perf}; do
    for v in new $VAR; do
      L=""; [ $v != new ] && L=$R/noise-c_amd/ab/libnoise_aead_hip_$v.so
      NOISE_AEAD_LIB=$L timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline ${EXTRA:-} > $O/${c}_${v}_$rep.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "import json;d=json.load(open('$O/${c}_${v}_$rep.json'));print('$c $v $rep',d['value'],d['roofline']['avg_launch_ms'],d.get('verified'))"
    done
  done
done

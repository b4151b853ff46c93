# A/B of the device kernels: noise-c_amd/ab/libnoise_aead_hip_prev.so (another
# build of the same ABI) against the current library, alternated on one box.
set -e
CFGS=${CFGS:-"c2 c4"}
for i in 1 2 3; do
 for v in prev new; do
  if [ $v = prev ]; then export NOISE_AEAD_LIB=$PWD/noise-c_amd/ab/libnoise_aead_hip_prev.so; else unset NOISE_AEAD_LIB; fi
  for c in $CFGS; do
   timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 | sed "s/}\$/, \"lib\": \"$v\"}/" >> gpurun_out/bench_ab.jsonl
  done
 done
done

# A/B of the host batch path: another build of the library
# (noise-c_amd/ab/libnoise_aead_hip_prev.so, same ABI) against the current one,
# alternated on one box because host-side rates drift between runs.
set -e
for i in 1 2 3 4; do
 for v in prev new; do
  if [ $v = prev ]; then
   export NOISE_AEAD_LIB=$PWD/noise-c_amd/ab/libnoise_aead_hip_prev.so
  else
   unset NOISE_AEAD_LIB
  fi
  for c in chachapoly aesgcm; do
   timeout -k 10 120 python tools/e2e.py --reps 10 --cipher $c | sed "s/}\$/, \"lib\": \"$v\"}/" >> gpurun_out/ab.jsonl
  done
 done
done

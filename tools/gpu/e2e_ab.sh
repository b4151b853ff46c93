# A/B of the host batch path: a previous build of the library (noise-c_amd/ab/,
# linked from the old cipherstate.c and the current objects) against the current one.
set -e
for i in 1 2 3 4; do
 for v in prev new; do
  if [ $v = prev ]; then export NOISE_AEAD_LIB=$PWD/noise-c_amd/ab/libnoise_aead_hip_prev.so  # built from the previous commit; else unset NOISE_AEAD_LIB; fi
  for c in chachapoly aesgcm; do
   timeout -k 10 120 python tools/e2e.py --reps 10 --cipher $c | sed "s/}\$/, \"lib\": \"$v\"}/" >> gpurun_out/ab.jsonl
  done
 done
done

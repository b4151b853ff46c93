# Single-record CipherState latency (tools/latency.c), zero-copy on and off.
set -e
mkdir -p gpurun_out
for zc in default 0; do
  for c in chachapoly aesgcm; do
    for n in 64 1024 4096 16384 65519; do
      if [ "$zc" = default ]; then
        timeout -k 10 60 ./tools/latency $c $n 2000 >> gpurun_out/latency.jsonl
      else
        NOISE_AEAD_ZERO_COPY_MAX=0 timeout -k 10 60 ./tools/latency $c $n 2000 | sed 's/}$/, "zero_copy": false}/' >> gpurun_out/latency.jsonl
      fi
    done
  done
done

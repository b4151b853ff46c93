# Worker latency, both ciphers, with the paths' cycle stamps.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_lat_aes; mkdir -p $O
: > $O/latency.jsonl
for c in aesgcm chachapoly; do
  for n in 64 1024 1400; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
cat $O/latency.jsonl

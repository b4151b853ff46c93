# Worker latency only (ChaChaPoly), with the latency-first path's cycle stamps.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_lat; mkdir -p $O
: > $O/latency.jsonl
for n in 64 256 1024 1400 2048 3000; do
  timeout -k 10 60 ./tools/latency chachapoly $n 2000 >> $O/latency.jsonl
done
cat $O/latency.jsonl

# GPU suite, then worker latency (both ciphers, stage stamps), then the doorbell microbench.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_aeslat; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
: > $O/latency.jsonl
for c in aesgcm chachapoly; do
  for n in 64 1024 1400; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
cat $O/latency.jsonl
timeout -k 10 60 ./tools/microbench/doorbell 5000 | tee $O/doorbell.jsonl

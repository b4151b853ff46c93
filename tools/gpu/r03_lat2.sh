# Worker + wide-record tests, AES block latency microbench, worker latency.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_lat2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 60 ./tools/microbench/aes_lat | tee $O/aes_lat.log
: > $O/latency.jsonl
for c in aesgcm chachapoly; do
  for n in 64 1024 1400 16384; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
cat $O/latency.jsonl

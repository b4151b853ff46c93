# Resident worker (single-record CipherState calls): latency first (bounded),
# then the GPU test suite with the worker on (default).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_worker; mkdir -p $O
: > $O/latency.jsonl
for w in 1 0; do
  for c in chachapoly aesgcm; do
    for n in 64 1024 16384 65519; do
      NOISE_AEAD_WORKER=$w timeout -k 10 60 ./tools/latency $c $n 2000 | sed "s/}\$/, \"worker\": $w}/" >> $O/latency.jsonl
    done
  done
done
cat $O/latency.jsonl
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log

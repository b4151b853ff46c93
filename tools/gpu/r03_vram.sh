# Worker with the request in device memory (default on a large-BAR device) vs host memory.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_vram; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py tests/test_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_worker.log 2>&1 || { tail -30 $O/pytest_worker.log; exit 1; }
tail -1 $O/pytest_worker.log
NOISE_AEAD_WORKER_VRAM=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_worker_host.log 2>&1 || { tail -30 $O/pytest_worker_host.log; exit 1; }
tail -1 $O/pytest_worker_host.log
: > $O/latency.jsonl
for v in 1 0; do
  for c in chachapoly aesgcm; do
    for n in 64 1024 1400 16384; do
      NOISE_AEAD_WORKER_VRAM=$v timeout -k 10 60 ./tools/latency $c $n 2000 | sed "s/}\$/, \"vram\": $v}/" >> $O/latency.jsonl
    done
  done
done
cat $O/latency.jsonl

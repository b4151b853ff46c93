# Round 5: the free-beside-concurrent-caller check with leave diagnostics,
# then the worker tests.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_wk2; mkdir -p $O
NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000 NOISE_AEAD_WORKER_QUEUES=2 NOISE_AEAD_WORKER_SLOTS=1 timeout -k 10 60 python -u tests/worker_mode_check.py --free-concurrent > $O/free_conc.txt 2>&1 || true
cat $O/free_conc.txt
NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000 timeout -k 10 60 python -u tests/worker_mode_check.py --free-check > $O/free_check.txt 2>&1 || true
cat $O/free_check.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -m gpu -v -x -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_worker.log 2>&1 || { tail -40 $O/pytest_worker.log; exit 1; }
grep -E "PASSED|FAILED|calls/s|memset" $O/pytest_worker.log | tail -20

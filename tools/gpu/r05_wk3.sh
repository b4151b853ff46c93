set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_wk3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -m gpu -v -x -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_worker.log 2>&1 || { tail -40 $O/pytest_worker.log; exit 1; }
grep -E "PASSED|FAILED|calls/s" $O/pytest_worker.log | tail -14

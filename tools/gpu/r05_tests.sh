# Round 5: the worker tests first (worker groups: several request slots per
# high-priority queue), then every other -m gpu test and smoke() on the
# current code, then the single-call thread scaling and the queue probe under
# the box's default queues.  Outputs in gpurun_out/r05_tests/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_tests}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -m gpu -v -x -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_worker.log 2>&1 || { tail -40 $O/pytest_worker.log; exit 1; }
tail -1 $O/pytest_worker.log
: > $O/mt_calls.txt
for c in chachapoly aesgcm; do for t in 1 2 4 8 12; do
  timeout -k 10 60 ./tools/mt_calls $c $t 1400 1.0 >> $O/mt_calls.txt 2>&1 || { tail -20 $O/mt_calls.txt; exit 1; }
done; done
cat $O/mt_calls.txt
if [ -z "${WORKER_ONLY:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --deselect tests/test_gpu_worker.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
echo done

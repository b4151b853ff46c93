# Correctness first, then a lanes-per-record sweep of bench.py (c2 unless given)
set -u
R=$GRAFT_REPO_ROOT; cd $R
CFG=${1:-c2}
if [ -z "${SKIP_TEST:-}" ]; then timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu.log; else rc=0; fi
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for k in ${LANES:-1 2 4 8}; do
  timeout -k 10 120 python bench.py --config $CFG --lanes $k --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/sweep_${CFG}_k$k.json 2> gpurun_out/sweep_${CFG}_k$k.err || { echo "bench k=$k failed"; tail -5 gpurun_out/sweep_${CFG}_k$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep_${CFG}_k$k.json'));print('K=$k value',d['value'],'seal',d['seal_gibs'],'open',d['open_gibs'],'frac',d['roofline']['frac'],'seal_ms',d['roofline']['avg_launch_ms'])"
done

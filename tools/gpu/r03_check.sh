# Round-3 check on MI355X: all GPU tests, then the default bench line (C2,
# with CPU baseline and verification) and C3.  Outputs in gpurun_out/r03_check/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r03_check}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_SEL:-} > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
echo done

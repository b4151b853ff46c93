# Session-2 check on MI355X: GPU tests, default bench line (C2) and C3, then
# the C2/C4-shape wave timeline (tools/microbench/timeline3).  Outputs in
# gpurun_out/r03_s2/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r03_s2}; mkdir -p $O
timeout -k 10 90 ./tools/microbench/aes_bs 20 > $O/aes_bs.log 2>&1 || { tail -20 $O/aes_bs.log; exit 1; }
cat $O/aes_bs.log
timeout -k 10 150 ./tools/microbench/timeline3 40 > $O/timeline3.log 2>&1 || { tail -20 $O/timeline3.log; exit 1; }
cat $O/timeline3.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
echo done

# Full round measurement: GPU parity, bench lines (C2 default with CPU baseline,
# C3, C4, C5, perf), end-to-end host paths (batch API, wire path, TCP echo),
# rocprofv3 kernel stats of the default bench.  Outputs in gpurun_out/round/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-round}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --steps 20 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 --verify > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
timeout -k 10 200 python bench.py --config perf > $O/bench_perf.json 2> $O/bench_perf.err || { tail -20 $O/bench_perf.err; exit 1; }
cat $O/bench_c3.json $O/bench_c4.json $O/bench_c5.json $O/bench_perf.json
timeout -k 10 300 python tools/e2e.py > $O/e2e_c2.json 2> $O/e2e_c2.err || { tail -20 $O/e2e_c2.err; exit 1; }
timeout -k 10 300 python tools/e2e.py --cipher aesgcm > $O/e2e_c3.json 2> $O/e2e_c3.err || { tail -20 $O/e2e_c3.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py > $O/wire_c2.jsonl 2> $O/wire_c2.err || { tail -20 $O/wire_c2.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py --cipher aesgcm > $O/wire_c3.jsonl 2> $O/wire_c3.err || { tail -20 $O/wire_c3.err; exit 1; }
timeout -k 10 300 python tools/echo_loopback.py > $O/echo.json 2> $O/echo.err || { tail -20 $O/echo.err; exit 1; }
cat $O/e2e_c2.json $O/e2e_c3.json $O/wire_c2.jsonl $O/wire_c3.jsonl $O/echo.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_c5.log 2>&1 || { tail -20 $O/prof_c5.log; exit 1; }
echo done

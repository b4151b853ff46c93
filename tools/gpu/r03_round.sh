# Round-3 measurement set on the final code: all GPU tests, smoke(), every
# bench line (C2 default with CPU baseline at the driver's --steps 20
# --warmup 5, C3, C4, C5, perf), worker latency, end-to-end host paths.
# Outputs in gpurun_out/r03_round/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_round; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json | cut -c1-400
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
timeout -k 10 300 python bench.py --config perf --steps 20 --warmup 5 > $O/bench_perf.json 2> $O/bench_perf.err || { tail -20 $O/bench_perf.err; exit 1; }
for c in c3 c4 c5 perf; do python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('cpu_baseline',{}).get('value'))"; done
: > $O/latency.jsonl
for c in chachapoly aesgcm; do
  for n in 64 1024 1400 16384 65519; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
timeout -k 10 300 python tools/e2e.py > $O/e2e_c2.json 2> $O/e2e_c2.err || { tail -20 $O/e2e_c2.err; exit 1; }
timeout -k 10 300 python tools/e2e.py --cipher aesgcm > $O/e2e_c3.json 2> $O/e2e_c3.err || { tail -20 $O/e2e_c3.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py > $O/wire_c2.jsonl 2> $O/wire_c2.err || { tail -20 $O/wire_c2.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py --cipher aesgcm > $O/wire_c3.jsonl 2> $O/wire_c3.err || { tail -20 $O/wire_c3.err; exit 1; }
timeout -k 10 300 python tools/echo_loopback.py > $O/echo.json 2> $O/echo.err || { tail -20 $O/echo.err; exit 1; }
echo done

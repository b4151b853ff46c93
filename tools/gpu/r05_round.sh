# Round-5 measurement set on the final code: all GPU tests, smoke(), every
# bench line at the driver's --steps 20 --warmup 5 (C2 default and C4 with
# their CPU baselines, C3, C5, perf), the verify-first open order's C2/C3
# lines, the one-rank RCCL lines (--rccl), worker latency and thread scaling, end-to-end host paths.
# Outputs in gpurun_out/r05_round/.  PART=1: tests, smoke, bench lines;
# PART=2: latency, thread scaling, host paths (unset: both).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_round}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ] && [ "${PART:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -x --durations=10 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if [ "${PART:-1}" = 1 ]; then
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('verified'),d['config'].get('open_order'),(d.get('cpu_baseline') or {}).get('value'))"
}
b c2 --steps 20 --warmup 5
b c3 --config c3 --steps 20 --warmup 5
b c4 --config c4 --steps 20 --warmup 5
b c5 --config c5 --steps 20 --warmup 5
b perf --config perf --steps 20 --warmup 5
b c2_verify_first --steps 20 --warmup 5 --verify-first --no-cpu-baseline
b c3_verify_first --config c3 --steps 20 --warmup 5 --verify-first --no-cpu-baseline
b c5_verify_first --config c5 --steps 10 --warmup 2 --verify-first --no-cpu-baseline
b c2_rccl --steps 20 --warmup 5 --rccl --no-cpu-baseline
b c5_rccl --config c5 --steps 20 --warmup 5 --rccl --no-cpu-baseline
timeout -k 10 300 python bench.py > $O/bench_default_noflags.json 2> $O/bench_default_noflags.err || { tail -20 $O/bench_default_noflags.err; exit 1; }
fi
if [ "${PART:-2}" = 2 ]; then
: > $O/latency.jsonl
for c in chachapoly aesgcm; do
  for n in 64 1024 1400 16384 65519; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
: > $O/mt_calls.txt
for c in chachapoly aesgcm; do for t in 1 2 4 8; do
  timeout -k 10 60 ./tools/mt_calls $c $t 1400 1.0 >> $O/mt_calls.txt 2>&1 || { tail -20 $O/mt_calls.txt; exit 1; }
done; done
timeout -k 10 300 python tools/e2e.py > $O/e2e_c2.json 2> $O/e2e_c2.err || { tail -20 $O/e2e_c2.err; exit 1; }
timeout -k 10 300 python tools/e2e.py --cipher aesgcm > $O/e2e_c3.json 2> $O/e2e_c3.err || { tail -20 $O/e2e_c3.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py > $O/wire_c2.jsonl 2> $O/wire_c2.err || { tail -20 $O/wire_c2.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py --cipher aesgcm > $O/wire_c3.jsonl 2> $O/wire_c3.err || { tail -20 $O/wire_c3.err; exit 1; }
timeout -k 10 300 python tools/echo_loopback.py > $O/echo.json 2> $O/echo.err || { tail -20 $O/echo.err; exit 1; }
fi
echo done

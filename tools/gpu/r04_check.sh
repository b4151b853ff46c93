# Round-4 check on MI355X: all GPU tests (or PYTEST_SEL), then bench lines
# for CFGS (default c2) with the driver's --steps 20 --warmup 5.
# Outputs in gpurun_out/${ROUND_DIR:-r04_check}/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_check}; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest ${PYTEST_SEL:-tests/} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
fi
for cfg in ${CFGS:-c2}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$cfg.json'));print('$cfg',d['value'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d['roofline']['kernel'],d.get('verified'),(d.get('cpu_baseline') or {}).get('value'))"
done
echo done

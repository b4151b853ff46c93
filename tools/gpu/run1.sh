set -u
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --verify > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo bench_fail; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 2 --verify > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo bench3_fail; tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
for k in 1 2 8; do timeout -k 10 120 python bench.py --lanes $k --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_c2_k$k.json 2>&1 || exit 1; cat gpurun_out/bench_c2_k$k.json | python -c "import json,sys;d=json.load(sys.stdin);print('K',$k,d['value'],d['seal_gibs'],d['open_gibs'],d['roofline']['frac'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/gpurun_out/prof_c2.log 2>&1; echo prof_rc=$?
ls -R $R/gpurun_out/prof_c2 | head

# GPU parity (uniform/duplex/staged subsets + full-size digests), then the C2 A/B of modes.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_check; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_config_digests.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit $rc; fi
for i in 1 2; do
  for m in duplex separate; do
    timeout -k 10 120 python bench.py --mode $m --no-cpu-baseline --steps 50 --warmup 10 --verify > $O/$m.$i.json 2> $O/$m.$i.err || { tail -20 $O/$m.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$m.$i.json'));print('$m',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d['seal_gibs'],d['open_gibs'],d.get('verified'))"
  done
done

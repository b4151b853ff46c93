# AES-GCM duplex launch: duplex parity tests, then C3 duplex vs separate
# (interleaved, --verify).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_aesdup; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "duplex or staged or in_place" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for m in duplex separate; do
    timeout -k 10 120 python bench.py --config c3 --mode $m --no-cpu-baseline --steps 40 --warmup 8 --verify > $O/c3.$m.$i.json 2> $O/c3.$m.$i.err || { tail -20 $O/c3.$m.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c3.$m.$i.json'));r=d['roofline'];print('$m',d['value'],d['ms_per_step'],r['kernel'],r['avg_launch_ms'],r['frac'],d['seal_gibs'],d['open_gibs'],d.get('verified'))"
  done
done
echo aesdup done

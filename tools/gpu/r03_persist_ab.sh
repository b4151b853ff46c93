# A/B of the persistent duplex kernel (NOISE_AEAD_DUPLEX=persist) against the
# per-workgroup duplex launch, interleaved on one box; parity first.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_persist_ab; mkdir -p $O
NOISE_AEAD_DUPLEX=persist timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k duplex tests/test_config_digests.py > $O/pytest_persist.log 2>&1 || { tail -40 $O/pytest_persist.log; exit 1; }
tail -1 $O/pytest_persist.log
for i in 1 2 3; do
  for m in plain persist; do
    for c in c2 perf; do
      NOISE_AEAD_DUPLEX=$m timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/$c.$m.$i.json 2> $O/$c.$m.$i.err || { tail -20 $O/$c.$m.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.$m.$i.json'));print('$c $m $i',d['value'],d['roofline']['avg_launch_ms'],d['verified'])"
    done
  done
done
for m in plain persist; do
  NOISE_AEAD_DUPLEX=$m timeout -k 10 200 python bench.py --config c4 --steps 20 --no-cpu-baseline > $O/c4.$m.json 2> $O/c4.$m.err || { tail -20 $O/c4.$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4.$m.json'));print('c4 $m',d['value'],d['roofline']['avg_launch_ms'],d['verified'])"
done
echo done

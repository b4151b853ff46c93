# Round-2 iteration: GPU suite, then library A/B (VARIANTS, CFGS), then the
# AES-GCM bench lines and C3 HBM-traffic passes of the current build.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_step; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider ${PYK:+-k "$PYK"} > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; fi
fi
if [ -n "${VARIANTS:-}" ]; then
  VARIANTS="$VARIANTS" CFGS="${CFGS:-c2}" ROUNDS=${ROUNDS:-2} bash tools/gpu/ab_libs.sh || exit 1
fi
for c in ${BENCH:-}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 20 > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  cut -c1-300 $O/$c.json; python3 -c "import json;d=json.load(open('$O/$c.json'));print({k:d.get(k) for k in ('value','seal_gibs','open_gibs','kernels_ms')})"
done
cd /tmp && export TMPDIR=/tmp
for c in ${PMC:-}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_$c/$ctr -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 ${PMC_ARGS:-} > $O/pmc_$c.$ctr.log 2>&1 || { echo "pmc $c $ctr failed"; tail -5 $O/pmc_$c.$ctr.log; exit 1; }
  done
done
echo step done

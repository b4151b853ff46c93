# Full GPU suite, then C2/C4 benches with the single-pass open.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_open1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; fi
for c in c2 c4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.err || exit 1
  cut -c1-200 $O/$c.json; grep -o '"seal_gibs[^}]*' $O/$c.json | cut -c1-120
done

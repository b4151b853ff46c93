# Full GPU test suite (one pytest process).  PYK="expr" selects with -k.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_tests; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider ${PYK:+-k "$PYK"} ${PYARGS:-} > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; fi
exit $rc

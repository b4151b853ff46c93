# CT-GHASH parity + pad/hardening tests, then C3 with and without the flag.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_ct; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ct_ghash.py tests/test_gpu_pad.py tests/test_gpu_hardening.py \
    -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --ct-ghash > $O/c3_ct.json 2> $O/c3_ct.err
rc=$?; cat $O/c3.json $O/c3_ct.json | cut -c1-400; exit $rc

# Round 5: find the GPU test that went silent in the full run (r05_round3):
# the parity tests before it and the RCCL file, verbose, to a file.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_hang; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py -m gpu -v -x --durations=15 --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -30 $O/pytest.log
exit $rc

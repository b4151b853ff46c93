# Parity of the wide-group Poly1305 tree (K >= 16, one step), the worker's
# latency and clock, then the settle A/B (tools/gpu/r03_settle.sh).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_s3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_verify_first.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/latency.jsonl
for c in chachapoly aesgcm; do
  for n in 64 1024 16384; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
cat $O/latency.jsonl
bash tools/gpu/r03_settle.sh

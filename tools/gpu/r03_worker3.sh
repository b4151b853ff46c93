# Worker with stamped-chunk speculative input: tests + latency; then the C3
# PMC passes on the fused AES-GCM duplex kernel (traffic_c3.json).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_worker3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_dropin.py tests/test_echo_dropin.py tests/test_gpu_hardening.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/latency.jsonl
for c in chachapoly aesgcm; do
  for n in 64 1024 1400 4096 16384 65519; do
    timeout -k 10 60 ./tools/latency $c $n 2000 >> $O/latency.jsonl
  done
done
cat $O/latency.jsonl
true
true

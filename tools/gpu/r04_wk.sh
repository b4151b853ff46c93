# Round 4: resident-worker tests (multi-pass ChaChaPoly, row GHASH) and
# single-record latency points for ChaChaPoly / AES-GCM.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_wk}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_worker.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_worker.log 2>&1 || { tail -40 $O/pytest_worker.log; exit 1; }
tail -3 $O/pytest_worker.log
for c in chachapoly aesgcm; do
  for n in 64 1024 1400 16384 65519; do
    timeout -k 10 60 ./tools/latency $c $n 2000 > $O/lat_${c}_$n.txt 2>&1 || { cat $O/lat_${c}_$n.txt; exit 1; }
    echo "$c $n: $(tail -2 $O/lat_${c}_$n.txt | tr '\n' ' ')"
  done
done
echo done

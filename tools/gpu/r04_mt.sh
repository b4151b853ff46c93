# Round 4: single-call throughput over threads (tools/mt_calls) with the
# worker's idle-poll backoff (default) and without it (variant library
# built with NA_POLL_BACKOFF far beyond the worker lifetime), interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_mt}; mkdir -p $O
: > $O/mt.txt
for rep in 1 2; do
  for v in default nb; do
    for c in chachapoly aesgcm; do
      for t in 1 2 4 8; do
        if [ $v = nb ]; then
          LD_LIBRARY_PATH=$R/noise-c_amd/ab/nb timeout -k 10 60 ./tools/mt_calls $c $t 1400 1.0 > $O/one.txt 2>&1 || { cat $O/one.txt; exit 1; }
        else
          timeout -k 10 60 ./tools/mt_calls $c $t 1400 1.0 > $O/one.txt 2>&1 || { cat $O/one.txt; exit 1; }
        fi
        echo "$v rep$rep $(cat $O/one.txt)" | tee -a $O/mt.txt
      done
    done
  done
done

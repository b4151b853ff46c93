# Round 5: worker groups — the free-beside-concurrent-caller check with its
# relaunch causes, then single-call latency and 1/8-thread call rates with
# the default groups (3 queues x 3 slots) against one slot per queue (the
# round-4 shape).  Outputs in gpurun_out/r05_wk/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_wk}; mkdir -p $O
NOISE_AEAD_DEBUG_WORKER_IDLE_MS=10000 NOISE_AEAD_WORKER_QUEUES=2 NOISE_AEAD_WORKER_SLOTS=1 timeout -k 10 60 python -u tests/worker_mode_check.py --free-concurrent > $O/free_conc.txt 2>&1 || true
cat $O/free_conc.txt
: > $O/lat.txt
for shape in default old; do
  if [ $shape = old ]; then export NOISE_AEAD_WORKER_QUEUES=4 NOISE_AEAD_WORKER_SLOTS=1; fi
  for n in 64 1400 16384; do
    echo "$shape $(timeout -k 10 60 ./tools/latency chachapoly $n 2000)" >> $O/lat.txt
  done
  echo "$shape $(timeout -k 10 60 ./tools/latency aesgcm 1400 2000)" >> $O/lat.txt
  for t in 1 8; do
    echo "$shape $(timeout -k 10 60 ./tools/mt_calls chachapoly $t 1400 1.0)" >> $O/lat.txt
  done
done
cat $O/lat.txt
echo done

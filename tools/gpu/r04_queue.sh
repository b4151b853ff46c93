# Round 4: resident single-call workers vs the device's hardware queues
# (GPU_MAX_HW_QUEUES, 4 on the pool): a memset on each newly created stream
# beside 1 / 4 busy workers, and mt_calls over threads, for the worker
# stream at normal (default), high and low priority.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_queue}; mkdir -p $O
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for p in normal high low; do
  for w in 1 4; do
    echo "prio=$p workers=$w $(NOISE_AEAD_WORKER_PRIO=$p timeout -k 10 60 ./tools/queue_probe 8 $w)"
  done
  for t in 4 8; do
    echo "prio=$p $(NOISE_AEAD_WORKER_PRIO=$p timeout -k 10 60 ./tools/mt_calls chachapoly $t 1400 1.0)"
  done
done

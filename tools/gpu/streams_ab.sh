# bench.py --streams 1 vs 2 (consecutive steps on alternating streams), one box.
set -e
for i in 1 2 3; do
 for n in 1 2; do
  for c in ${CFGS:-c2 c3 c4}; do
   timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --streams $n >> gpurun_out/streams_ab.jsonl
  done
 done
done

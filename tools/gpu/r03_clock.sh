# Clock of the C2-shaped duplex launch vs warm-up length and launch size
# (tools/microbench/timeline3): is C2's deficit against C4 the clock?
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_clock; mkdir -p $O
: > $O/clock.log
for w in 10 200 2000; do
  echo "== warm $w, C2 shape only" >> $O/clock.log
  timeout -k 10 120 ./tools/microbench/timeline3 $w 65536 0 >> $O/clock.log 2>&1
done
echo "== warm 40, C4 shape first, then C2 shape" >> $O/clock.log
timeout -k 10 120 ./tools/microbench/timeline3 40 0 0 1 >> $O/clock.log 2>&1
cat $O/clock.log

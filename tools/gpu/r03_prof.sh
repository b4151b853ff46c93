# rocprofv3 kernel-trace summaries of the round-3 bench lines: C2 (default,
# the driver's --steps 20 --warmup 5, settled), C3, and C5 with its two
# kernel families on ONE stream (--c5-streams 1: the summary's averages are
# the serial per-kernel times the C5 line's kernels_ms quotes).
set -eu
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2> $O/prof_c2.log || { tail -20 $O/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2> $O/prof_c3.log || { tail -20 $O/prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --c5-streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_serial.json 2> $O/prof_c5.log || { tail -20 $O/prof_c5.log; exit 1; }
for c in c2 c3 c5; do
  f=$(find $O/prof_$c -name '*kernel_stats.csv' | head -1)
  echo "== $c $f"; head -8 "$f" | cut -c1-200
done
cat $O/bench_c2.json $O/bench_c3.json $O/bench_c5_serial.json | cut -c1-300

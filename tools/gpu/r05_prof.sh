# Round 5: rocprofv3 --kernel-trace --stats of the bench lines (C2, C3 at
# the driver's --steps 20 --warmup 5; C5 serial), then the statistics of the
# TIMED dispatches only (tools/kernel_window.py: the last --steps dispatches
# of the step kernel) beside rocprof's whole-run summary.  Each profiled
# run's own bench line is kept with it.  Outputs in gpurun_out/r05_prof/.
set -eu
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${ROUND_DIR:-r05_prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() {  # name substr steps bench-args...
  local n=$1 sub=$2 k=$3; shift 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 $R/bench.py --steps $k "$@" --no-cpu-baseline > $O/bench_${n}_profiled.json 2> $O/prof_$n.log || { tail -20 $O/prof_$n.log; exit 1; }
  cp $(find $O/prof_$n -name '*kernel_stats.csv' | head -1) $O/${n}_kernel_stats_all.csv
  python3 $R/tools/kernel_window.py $O/prof_$n "$sub" $k $O/${n}_kernel_stats_timed.csv
  python3 -c "import json;d=json.load(open('$O/bench_${n}_profiled.json'));print('$n line',d['value'],'ms_per_step',d['ms_per_step'],'launch_ms',d['roofline']['avg_launch_ms'],'frac',d['roofline']['frac'],d.get('verified'))"
}
prof c2 duplex 20 --warmup 5
prof c3 duplex 20 --warmup 5 --config c3
prof c4 duplex 20 --warmup 5 --config c4
prof perf duplex 20 --warmup 5 --config perf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --c5-streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_serial_profiled.json 2> $O/prof_c5.log || { tail -20 $O/prof_c5.log; exit 1; }
cp $(find $O/prof_c5 -name '*kernel_stats.csv' | head -1) $O/c5_kernel_stats_all.csv
head -8 $O/c5_kernel_stats_all.csv | cut -c1-160
# the default two-stream step's trace: the halves overlapping (tools/c5_timeline.py)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5_step -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5_profiled.json 2> $O/prof_c5_step.log || { tail -20 $O/prof_c5_step.log; exit 1; }
python3 $R/tools/c5_timeline.py $O/prof_c5_step 5 > $O/c5_timeline.txt
tail -1 $O/c5_timeline.txt
echo done

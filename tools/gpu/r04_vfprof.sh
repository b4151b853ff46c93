# Round 4: kernel trace of the C2 bench line with the verify-first open vs
# one pass (which kernels run, their timed-window durations), and the
# timeline microbenchmark beside it.
set -eu
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${ROUND_DIR:-r04_vfprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for vf in 0 1; do
  F=""; [ $vf = 1 ] && F="--verify-first"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vf$vf -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline $F > $O/bench_vf$vf.json 2> $O/prof_vf$vf.log || { tail -20 $O/prof_vf$vf.log; exit 1; }
  python3 $R/tools/kernel_window.py $O/prof_vf$vf duplex 20 $O/timed_vf$vf.csv
  cp $(find $O/prof_vf$vf -name '*kernel_stats.csv' | head -1) $O/all_vf$vf.csv
  head -4 $O/all_vf$vf.csv | cut -c1-150
  python3 -c "import json;d=json.load(open('$O/bench_vf$vf.json'));print('vf=$vf line',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
cd $R/tools/microbench && timeout -k 10 60 ./timeline_solo 1 256 400 4 | head -2

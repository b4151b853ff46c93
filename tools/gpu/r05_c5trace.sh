# Round 5: kernel trace of the C5 step (two streams, one join per step):
# which kernels overlap, the step span against the kernel sum.
set -eu
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r05_c5trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --config c5 --no-cpu-baseline --settle-ms 200 --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err
python3 $R/tools/c5_timeline.py $O/trace 3 > $O/timeline.txt
cat $O/timeline.txt

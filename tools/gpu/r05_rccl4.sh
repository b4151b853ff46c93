# Round 5: kernel traces of C5 with and without the one-rank RCCL group:
# which hardware queue each dispatch used.  gpurun_out/r05_rccl4/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_rccl4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config c5 --steps 5 --warmup 2 --settle-ms 0 --no-cpu-baseline --no-verify --no-xfer"
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/plain -o run --output-format csv -- python3 $B > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/rccl -o run --output-format csv -- python3 $B --rccl > $O/rccl.json 2> $O/rccl.err || exit 1
find $O -name "*kernel_trace.csv" | head

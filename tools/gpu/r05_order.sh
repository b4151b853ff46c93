# Round 5: C5 with the ChaChaPoly half launched first (its plan kernels and
# persistent seal take the CUs before the CU-exclusive AES-GCM windows)
# against AES-GCM first, interleaved; then the kernel trace of the faster.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_order}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d.get('verified'))"
}
for r in 1 2 3; do
b c5_aes_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
b c5_chacha_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline --c5-first chacha
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --config c5 --no-cpu-baseline --settle-ms 200 --steps 10 --warmup 2 --c5-first chacha > $O/trace_bench.json 2> $O/trace_bench.err
python3 $R/tools/c5_timeline.py $O/trace 2

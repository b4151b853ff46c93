# Round 5: C5 with each cipher's open after its own seal (--c5-join step,
# the new default) against both seals before either open (phase),
# interleaved.  Outputs in gpurun_out/r05_join/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_join}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('kernels_ms'))"
}
for r in 1 2 3; do
b c5_step_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
b c5_phase_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline --c5-join phase
done
echo done

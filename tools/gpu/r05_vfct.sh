# Round 5: the costs VERDICT r4 asks to re-measure on the final kernels:
# C3 with the constant-time GHASH (--ct-ghash) against the table GHASH, and
# C2 with the reference's open order (--verify-first) against one pass,
# interleaved.  Outputs in gpurun_out/r05_vfct/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_vfct}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d.get('verified'))"
}
for r in 1 2; do
b c3_tab_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
b c3_ct_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline --ct-ghash
b c2_onepass_$r --steps 20 --warmup 5 --no-cpu-baseline
b c2_vf_$r --steps 20 --warmup 5 --no-cpu-baseline --verify-first
done
echo done

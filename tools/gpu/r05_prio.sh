# Round 5: C5 (--c5-join step) with the AES-GCM or the ChaChaPoly half on a
# high-priority stream, against neither, interleaved.  gpurun_out/r05_prio/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_prio}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d.get('verified'))"
}
for r in 1 2; do
b c5_none_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
b c5_aes_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline --c5-prio aes
b c5_chacha_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline --c5-prio chacha
done
echo done

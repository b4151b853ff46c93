# Round 4: verify-first ChaChaPoly with the AUTH pass at top priority vs the
# one-pass default, interleaved (C2, C4, perf duplex lines; C5 mixed).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_vf3}; mkdir -p $O
run() {  # tag bench-args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -20 $O/$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),'seal',d.get('seal_gibs'),'open',d.get('open_gibs'),d.get('kernels_ms'))"
}
for rep in 1 2; do
  for c in c2 c4 perf; do
    run ${c}_vf0_$rep --config $c --steps 20 --warmup 5
    run ${c}_vf1_$rep --config $c --steps 20 --warmup 5 --verify-first
  done
  run c5_vf0_$rep --config c5 --steps 10 --warmup 2
  run c5_vf1_$rep --config c5 --steps 10 --warmup 2 --verify-first
done
echo done

# Round 4: standalone seal/open launches (bench --mode separate: the step is
# a seal launch and an open launch) at one lane vs four lanes per record,
# interleaved, C2 and C4; plus the default (library's choice).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_sep}; mkdir -p $O
run() {  # tag bench-args...
  local t=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --mode separate --steps 20 --warmup 5 "$@" > $O/$t.json 2> $O/$t.err || { tail -20 $O/$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['kernel'],d.get('verified'))"
}
for rep in 1 2; do
  for c in c2 c4; do
    run ${c}_k1_$rep --config $c --lanes 1
    run ${c}_k4_$rep --config $c --lanes 4
    run ${c}_auto_$rep --config $c
  done
done

# The bench with and without the sustained-load settle phase, at the driver's
# --steps 20 --warmup 5, interleaved; then C3, C4, C5 with it.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_settle; mkdir -p $O
: > $O/ab.jsonl
for i in 1 2; do
  for ms in 0 500; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --settle-ms $ms --no-cpu-baseline > $O/c2.$ms.$i.json 2> $O/c2.$ms.$i.err || { tail -20 $O/c2.$ms.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2.$ms.$i.json'));print(json.dumps({'settle_ms':$ms,'i':$i,'value':d['value'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac'],'issue':d['roofline']['issue_bound']['frac'],'settle':d['config']['settle'],'verified':d['verified']}))" | tee -a $O/ab.jsonl
  done
done
for c in c3 c4 c5 perf; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$c.json'));print('$c',d['value'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d.get('verified'))"
done
echo done

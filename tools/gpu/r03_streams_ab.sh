# Duplex steps on one stream vs alternating over two, interleaved, at the
# driver's command shape (C2, C3, perf); verification on.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_streams; mkdir -p $O
: > $O/ab.jsonl
for i in 1 2 3; do
  for c in c2 c3 perf; do
    for n in 1 2; do
      timeout -k 10 200 python bench.py --config $c --streams $n --steps 20 --warmup 5 --no-cpu-baseline > $O/$c.$n.$i.json 2> $O/$c.$n.$i.err || { tail -20 $O/$c.$n.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.$n.$i.json'));print(json.dumps({'config':'$c','streams':$n,'i':$i,'value':d['value'],'launch_ms':d['roofline']['avg_launch_ms'],'verified':d['verified']}))" | tee -a $O/ab.jsonl
    done
  done
done

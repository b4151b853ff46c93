# 16-B vs 128-B record slots (bench --align), every uniform config, three
# interleaved rounds on one box.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_align_all; mkdir -p $O
for i in 1 2 3; do
  for c in c2 c3 c4 perf; do
    for a in 16 128; do
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 8 --align $a --verify > $O/$c.a$a.$i.json 2> $O/$c.a$a.$i.err || { tail -20 $O/$c.a$a.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.a$a.$i.json'));print('$c align $a',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'))"
    done
  done
done
echo align_all done

# 128-B record slots (bench --align 128) vs the default 16: C2/C4 speed,
# interleaved, then the HBM-traffic passes of C2 at 128.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_align128; mkdir -p $O
for i in 1 2; do
  for c in c2 c4; do
    for a in 16 128; do
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 8 --align $a > $O/$c.a$a.$i.json 2> $O/$c.a$a.$i.err || { tail -20 $O/$c.a$a.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.a$a.$i.json'));print('$c align $a',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],'seal',d['seal_gibs'],'open',d['open_gibs'])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_c2/$ctr -o run --output-format csv -- python3 $R/bench.py --config c2 --no-cpu-baseline --steps 10 --warmup 2 --align 128 > $O/pmc.$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/pmc.$ctr.log; exit 1; }
done
python3 $R/tools/pmc_report.py $O/pmc_c2 c2 $O/traffic_c2_a128.json | grep -E "chacha" | cut -c1-250
echo align128 done

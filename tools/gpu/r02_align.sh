# Record-slot alignment A/B (bench --align 16 vs 64), interleaved, then the
# HBM-traffic passes of C3 with 64-B slots.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_align; mkdir -p $O
for i in 1 2; do
  for c in ${CFGS:-c3 c2}; do
    for a in 16 64; do
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 8 --align $a > $O/$c.a$a.$i.json 2> $O/$c.a$a.$i.err || { tail -20 $O/$c.a$a.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.a$a.$i.json'));print('$c align $a',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],'seal',d['seal_gibs'],'open',d['open_gibs'])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for c in ${PMC:-c3}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_$c/$ctr -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 --align 64 > $O/pmc_$c.$ctr.log 2>&1 || { echo "pmc $c $ctr failed"; tail -5 $O/pmc_$c.$ctr.log; exit 1; }
  done
  python3 $R/tools/pmc_report.py $O/pmc_$c $c $O/traffic_${c}_a64.json | grep -E "gcm|chacha" | cut -c1-250
done
echo align done

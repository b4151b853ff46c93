# A/B of bench modes on one box (C2 by default): duplex vs separate x event placement.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/ab_modes; mkdir -p $O
CFG=${CFG:-c2}
for i in 1 2; do
  for m in duplex separate; do
   for e in ends step; do
    timeout -k 10 120 python bench.py --config $CFG --mode $m --events $e --no-cpu-baseline --steps 50 --warmup 10 --verify > $O/$m.$e.$i.json 2> $O/$m.$e.$i.err || { tail -20 $O/$m.$e.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$m.$e.$i.json'));print('$m $e',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d['seal_gibs'],d['open_gibs'],d.get('verified'))"
   done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 50 --warmup 10 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cd $R && python3 tools/kgaps.py $O/kt chachapoly
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kts -o run --output-format csv -- python3 $R/bench.py --config $CFG --mode separate --no-cpu-baseline --steps 50 --warmup 10 > $O/kts.log 2>&1 || { tail -20 $O/kts.log; exit 1; }
cd $R && python3 tools/kgaps.py $O/kts chachapoly

# Round-2 probe: baseline C2 bench on this box + kernel trace (inter-kernel gaps).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_probe; mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 50 --warmup 10 > $O/kt_c2.log 2>&1 || { tail -20 $O/kt_c2.log; exit 1; }
cd $R && python3 tools/kgaps.py $O/kt_c2 chachapoly

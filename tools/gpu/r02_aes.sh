# GPU parity subset + C3/C5 bench + write/fetch PMC of the AES kernels.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_aes; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit $rc; fi
for c in c3 c5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 4 --verify > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d.get('seal_gibs'),d.get('open_gibs'),d.get('kernels_ms'),d.get('verified', d.get('all_tags_verified')))"
done
cd /tmp && export TMPDIR=/tmp
for c in c3 c5; do
  n=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
    n=$((n+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc_$c/p$n -o run --output-format csv -- python3 $R/bench.py --config $c --mode separate --no-cpu-baseline --steps 6 --warmup 2 > $O/pmc_$c.p$n.log 2>&1 || { echo "pmc $c $grp failed"; tail -5 $O/pmc_$c.p$n.log; }
  done
  python3 $R/tools/pmc_report.py $O/pmc_$c $c $O/traffic_$c.json
done

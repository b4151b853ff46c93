# Round-2 state check: GPU suite, bench lines C2 (with CPU baseline), C3, C4, C5,
# rocprofv3 kernel stats of the default C2 bench.  Outputs in gpurun_out/r02_state/.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_state; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cat $O/c2.json
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 20 > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  cut -c1-400 $O/$c.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
echo done

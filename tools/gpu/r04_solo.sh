# Round 4: one-lane-per-record ChaChaPoly kernels (seal_solo_staged) —
# parity subset, then interleaved C2/C4/perf A/B against the 4-lane kernels.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_solo}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${PYTEST_K:-staged_kernels or duplex or in_place or uniform_seal_open or with_ad or max_record}" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for rep in 1 2; do
  for cfg in ${CFGS:-c2 c4 perf}; do
    for k in 4 1; do
      timeout -k 10 200 python bench.py --config $cfg --lanes $k --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${cfg}_k${k}_$rep.json 2> $O/b_${cfg}_k${k}_$rep.err || { tail -20 $O/b_${cfg}_k${k}_$rep.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$O/b_${cfg}_k${k}_$rep.json')); print('$cfg k=$k rep $rep', d['value'], d.get('verified'), d.get('roofline',{}).get('frac'))"
    done
  done
done
echo done

# Round 4: chachapoly_duplex_solo's seal/open block placement — runs of the
# CU count (default) vs block-by-block alternation (NOISE_AEAD_DUPLEX_RUNS=0),
# interleaved, three rounds.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_runs}; mkdir -p $O
for rep in 1 2 3; do
  for c in c2 c4 perf; do
    for v in runs alt; do
      E=X=1; [ $v = alt ] && E=NOISE_AEAD_DUPLEX_RUNS=0
      env $E timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${c}_${v}_$rep.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      python3 -c "import json;d=json.load(open('$O/${c}_${v}_$rep.json'));print('$c $v $rep',d['value'],d['roofline']['avg_launch_ms'],d.get('verified'))"
    done
  done
done

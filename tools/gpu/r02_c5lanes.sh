# C5: lanes per ChaChaPoly record in the ragged kernels (library default 4
# at 64 Ki records) vs 8 and 16, interleaved, --verify.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_c5lanes; mkdir -p $O
for i in 1 2; do
  for k in 0 8 16; do
    timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 4 --lanes $k --verify > $O/c5.k$k.$i.json 2> $O/c5.k$k.$i.err || { tail -20 $O/c5.k$k.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5.k$k.$i.json'));print('k$k',d['value'],d['ms_per_step'],d['kernels_ms'],d['all_tags_verified'])"
  done
done
echo c5lanes done

# The N>1 path of bench.py end to end on a one-GPU box: --gpus 2 starts its
# own two ranks (gloo, both on GPU 0: NOISE_BENCH_REHEARSE=1), settle,
# timed steps, verification, the in-run N=1 reference, scatter/gather leg.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_rehearse; mkdir -p $O
NOISE_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --settle-ms 200 > $O/c2_2rank.json 2> $O/c2_2rank.err || { tail -30 $O/c2_2rank.err; exit 1; }
cut -c1-1500 $O/c2_2rank.json
NOISE_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --config c4 --steps 5 --warmup 1 --settle-ms 200 > $O/c4_2rank.json 2> $O/c4_2rank.err || { tail -30 $O/c4_2rank.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4_2rank.json'));print({k:d.get(k) for k in ('value','n_gpus','scaling','verified','per_gpu_efficiency','n1_in_run','rehearsal')})"

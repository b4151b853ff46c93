# Round 5: bench.py's N > 1 path on RCCL at one rank (tests/test_gpu_rccl.py)
# plus the two bench lines it checks.  Outputs in gpurun_out/r05_rccl/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_rccl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_rccl.log 2>&1 || { tail -60 $O/pytest_rccl.log; exit 1; }
tail -3 $O/pytest_rccl.log
for c in c2 c5; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --rccl --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -30 $O/bench_$c.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['process_group'],d['scatter_gather_ok'],d['scatter_gather'])"
done

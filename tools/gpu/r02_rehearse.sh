# N>1 code path rehearsal on a one-GPU box: 2 ranks on cuda:0 over gloo
# (NOISE_BENCH_REHEARSE=1), C2, C4 and C5, with the scatter/gather legs.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_rehearse; mkdir -p $O
for c in c2 c4 c5; do
  NOISE_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config $c --steps 6 --warmup 2 --n1-value 1000 > $O/rh_$c.json 2> $O/rh_$c.err || { tail -30 $O/rh_$c.err; exit 1; }
  grep '^{' $O/rh_$c.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$c',d['value'],d['n_gpus'],d.get('per_gpu_efficiency'),d.get('scatter_gather',{}).get('verified'),d.get('rehearsal','')[:40])"
done
echo rehearse done

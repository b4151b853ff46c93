# Round 5: what slows C5 under torchrun + RCCL (827 vs 964 GiB/s)?  C5 four
# ways: plain, torchrun without a group, --rccl without torchrun, torchrun
# --rccl with OMP_NUM_THREADS=16.  Outputs in gpurun_out/r05_rccl2/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_rccl2; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29517"
B="bench.py --gpus 1 --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-xfer"
b() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d.get('kernels_ms'),d.get('process_group'))"; }
for r in 1 2; do
b plain_$r python $B
b torchrun_$r $TR $B
b rccl_$r python $B --rccl
b torchrun_rccl_$r $TR $B --rccl
OMP_NUM_THREADS=16 b torchrun_rccl_omp_$r $TR $B --rccl
done

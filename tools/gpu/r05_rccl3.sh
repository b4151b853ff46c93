# Round 5: C5 with the process group after the C5 streams are made
# (bench.py C5_STREAMS), against the plain run.  gpurun_out/r05_rccl3/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_rccl3; mkdir -p $O
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29517"
B="bench.py --gpus 1 --config c5 --steps 20 --warmup 5 --no-cpu-baseline"
b() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d.get('kernels_ms'),d.get('process_group'),d.get('scatter_gather_ok'),d.get('verified'))"; }
for r in 1 2; do
b plain_$r python $B --no-xfer
b torchrun_rccl_$r $TR $B --rccl
done

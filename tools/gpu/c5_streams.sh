set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 150 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --c5-streams 1 >> gpurun_out/c5s.log 2>&1
  timeout -k 10 150 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --c5-streams 2 >> gpurun_out/c5s.log 2>&1
done
NOISE_BENCH_REHEARSE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --config c4 --no-cpu-baseline > gpurun_out/c4r.log 2>&1

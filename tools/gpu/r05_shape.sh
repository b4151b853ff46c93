# Round 5: C5 with the AES-GCM ragged windows at 4 lanes per record, 512
# records per window (NOISE_AEAD_GCM_SHAPE=w1024r2: 128 windows, the
# ChaChaPoly half filling the other CUs) against the default 8 lanes / 256
# records, interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_shape}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));k=d.get('kernels_ms');print('$n',d['value'],d['ms_per_step'],d.get('verified'),k)"
}
for r in 1 2 3; do
b c5_k8_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_GCM_SHAPE=w1024r2 b c5_k4_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

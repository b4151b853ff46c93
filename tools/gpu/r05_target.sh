# Round 5: SEG_TARGET (blocks per lane a ragged record aims at) A/B at C5:
# 32 (default) against 24, 48, 64 (ab/ variants), interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_target}; mkdir -p $O
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));k=d.get('kernels_ms');print('$n',d['value'],d['ms_per_step'],d.get('verified'),k['chacha_seal'],k['chacha_open'])"
}
for r in 1 2; do
b c5_t32_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
for t in 24 48 64; do
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_t$t.so b c5_t${t}_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
done
echo done

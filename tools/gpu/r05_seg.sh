# Round 5: the segmented one-lane ChaChaPoly kernels (chachapoly_seg.hip) —
# parity first (the new tests, the full-size digests incl. the standalone C2
# launches and the eight C5 shards), then the bench lines they change: the
# standalone 64 Ki seal/open (--mode separate, seal_gibs), C5, and C2 duplex
# unchanged.  Outputs in gpurun_out/r05_seg/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_seg}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_config_digests.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_seg.log 2>&1 || { tail -40 $O/pytest_seg.log; exit 1; }
tail -3 $O/pytest_seg.log
fi
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('seal_gibs'),d.get('open_gibs'),d.get('kernels_ms'))"
}
for r in 1 2; do
b sep_seg_$r --steps 20 --warmup 5 --mode separate --no-cpu-baseline
NOISE_AEAD_SEG=0 b sep_k4_$r --steps 20 --warmup 5 --mode separate --no-cpu-baseline
b c5_seg_$r --config c5 --steps 10 --warmup 2 --no-cpu-baseline
NOISE_AEAD_SEG=0 b c5_k8_$r --config c5 --steps 10 --warmup 2 --no-cpu-baseline
done
b c2 --steps 20 --warmup 5 --no-cpu-baseline
echo done

# Round 5: two interleaved CTR lookup chains per lane in the staged AES-GCM
# record (NA_GCM_X2=1, ab/libnoise_aead_hip_x2.so) against the default: the
# AES GPU tests on the variant, then C3 and C5 interleaved.
# Outputs in gpurun_out/r05_x2/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_x2; mkdir -p $O
X=$R/noise-c_amd/ab/libnoise_aead_hip_x2.so
NOISE_AEAD_LIB=$X timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x -k "aes or gcm" --deselect tests/test_gpu_worker.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('kernels_ms'))"
}
for r in 1 2; do
b c3_base_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b c3_x2_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
b c5_base_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b c5_x2_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

# Round 5: AES-GCM tag mask E_K(J0) in a spare GHASH slot (every AES-GCM
# staged/ragged kernel) against the previous build (ab/..._prev.so): all
# GPU tests but the worker's, then C3 and C5 interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_vslot}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --deselect tests/test_gpu_worker.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('kernels_ms'))"
}
for r in 1 2 3; do
b c3_new_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_prev.so b c3_prev_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
b c5_new_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_prev.so b c5_prev_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

# Round 5: AES-GCM round keys through the scalar cache (NA_RK_SCALAR, the
# default) against the LDS copy (ab/libnoise_aead_hip_rklds.so): every GPU
# test but the worker's on the default build, then C3 and C5 interleaved.
# Outputs in gpurun_out/r05_rk/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_rk}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --deselect tests/test_gpu_worker.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('kernels_ms'))"
}
for r in 1 2; do
b c3_sgpr_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_rklds.so b c3_lds_$r --config c3 --steps 20 --warmup 5 --no-cpu-baseline
b c5_sgpr_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_rklds.so b c5_lds_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

# Round 5: the verify-first AUTH pass with registers D steps deep
# (NA_AUTH_REG=D, default 3) against the LDS-tile pass (0): the GPU tests
# on the default build, then C2 --verify-first per variant and the one-pass
# line, interleaved.  Outputs in gpurun_out/r05_auth/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_auth}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --deselect tests/test_gpu_worker.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'))"
}
for r in 1 2; do
b c2_onepass_$r --steps 20 --warmup 5 --no-cpu-baseline
b c2_vf3_$r --steps 20 --warmup 5 --no-cpu-baseline --verify-first
for d in 0 2 4 6; do
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_auth$d.so b c2_vf${d}_$r --steps 20 --warmup 5 --no-cpu-baseline --verify-first
done
done
echo done

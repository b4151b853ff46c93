# Round 5: the verify-first DEC pass in reverse step order (NA_DEC_REV=1,
# ab/libnoise_aead_hip_decrev.so: the two steps the AUTH pass leaves in the
# tiles are not read again): every GPU test on the variant, then C2
# --verify-first and the one-pass C2 interleaved.  gpurun_out/r05_decrev/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_decrev; mkdir -p $O
X=$R/noise-c_amd/ab/libnoise_aead_hip_decrev.so
NOISE_AEAD_LIB=$X timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --deselect tests/test_gpu_worker.py --deselect tests/test_gpu_rccl.py --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'))"; }
for r in 1 2 3; do
b vf_base_$r python bench.py --config c2 --verify-first --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b vf_rev_$r python bench.py --config c2 --verify-first --steps 20 --warmup 5 --no-cpu-baseline
b c2_base_$r python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline
done

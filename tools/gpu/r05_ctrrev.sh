# Round 5: the AES-GCM verify-first CTR pass last block first
# (NA_GCM_CTR_REV=1, ab/libnoise_aead_hip_ctrrev.so) vs first block first:
# the AES GPU tests on the variant, then C3 and C5 interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_ctrrev; mkdir -p $O
X=$R/noise-c_amd/ab/libnoise_aead_hip_ctrrev.so
NOISE_AEAD_LIB=$X timeout -k 10 600 python -u -m pytest tests/ -m gpu -v -x -k "aes or gcm or c3 or c5 or dropin or hardening or cipherstate" --deselect tests/test_gpu_worker.py --deselect tests/test_gpu_rccl.py --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),d.get('kernels_ms'))"; }
for r in 1 2; do
b c3_base_$r python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b c3_rev_$r python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
b c5_base_$r python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b c5_rev_$r python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done

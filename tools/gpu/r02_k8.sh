# 8-lane paired AES-GCM windows: full GPU suite, the ragged tests under each
# forced shape, then C5 interleaved A/B (default = w1024r2k8 at N = 1).
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_k8; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; fi
for sh in w1024r1 w1024r2k8; do
  NOISE_AEAD_GCM_SHAPE=$sh timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ct_ghash.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "ragged" > $O/pytest_$sh.log 2>&1 || { tail -30 $O/pytest_$sh.log; exit 1; }
  tail -1 $O/pytest_$sh.log
done
for i in 1 2; do
  for sh in w1024r1 w1024r2k8; do
    NOISE_AEAD_GCM_SHAPE=$sh timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 > $O/c5.$sh.$i.json 2> $O/c5.$sh.$i.err || { tail -20 $O/c5.$sh.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5.$sh.$i.json'));print('$sh',d['value'],d['ms_per_step'],d['kernels_ms'],d['all_tags_verified'])"
  done
done
echo k8 done

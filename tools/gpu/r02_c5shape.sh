# Ragged AES-GCM launch shape (NOISE_AEAD_GCM_SHAPE): parity of each shape on
# the ragged tests, then C5 interleaved A/B of the shapes.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_c5shape; mkdir -p $O
for sh in w512r2 w1024r2; do
  NOISE_AEAD_GCM_SHAPE=$sh timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_config_digests.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "ragged or c5 or C5" > $O/pytest_$sh.log 2>&1 || { tail -30 $O/pytest_$sh.log; exit 1; }
  tail -1 $O/pytest_$sh.log
done
for i in 1 2; do
  for sh in w1024r1 w512r2 w1024r2; do
    NOISE_AEAD_GCM_SHAPE=$sh timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 > $O/c5.$sh.$i.json 2> $O/c5.$sh.$i.err || { tail -20 $O/c5.$sh.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5.$sh.$i.json'));print('$sh',d['value'],d['ms_per_step'],d['kernels_ms'],d['all_tags_verified'])"
  done
done
echo c5shape done

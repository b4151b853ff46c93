# A/B of the fused AES-GCM duplex kernel (NOISE_AEAD_GCM_DUPLEX=fused: one
# LDS fill, seal then open per workgroup) against gcm_duplex_staged;
# parity first (the duplex tests and the full-size digests under fused).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r03_gcm_fused; mkdir -p $O
NOISE_AEAD_GCM_DUPLEX=fused timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k duplex tests/test_config_digests.py > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
: > $O/ab.jsonl
for i in 1 2 3; do
  for m in staged fused; do
    NOISE_AEAD_GCM_DUPLEX=$m timeout -k 10 200 python bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline > $O/c3.$m.$i.json 2> $O/c3.$m.$i.err || { tail -20 $O/c3.$m.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c3.$m.$i.json'));print(json.dumps({'mode':'$m','i':$i,'value':d['value'],'launch_ms':d['roofline']['avg_launch_ms'],'verified':d['verified']}))" | tee -a $O/ab.jsonl
  done
done

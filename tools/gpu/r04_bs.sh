# Round 4: bitsliced-AES GCM kernels (NOISE_AEAD_GCM_BS=1) — AES parity
# subset under the switch, then interleaved C3 A/B (T-table vs bitsliced).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_bs}; mkdir -p $O
NOISE_AEAD_GCM_BS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config_digests.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${PYTEST_K:-(staged_kernels or in_place or duplex or full) and (AES or 17154 or c3 or 0-256 or slot128 or fast)}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
NOISE_AEAD_GCM_BS=2 timeout -k 10 600 python -u -m pytest tests/test_config_digests.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "c3" > $O/pytest_bs8.log 2>&1 || { tail -40 $O/pytest_bs8.log; exit 1; }
tail -3 $O/pytest_bs8.log
for rep in 1 2; do
  for v in 0 1 2; do
    NOISE_AEAD_GCM_BS=$v timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_bs${v}_$rep.json 2> $O/c3_bs${v}_$rep.err || { tail -20 $O/c3_bs${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c3_bs${v}_$rep.json'));print('bs=$v rep $rep',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),'seal',d['seal_gibs'],'open',d['open_gibs'])"
  done
done
echo done

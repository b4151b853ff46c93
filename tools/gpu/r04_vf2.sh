# Round 4: verify-first AUTH pass through registers (NOISE_AEAD_VF_AUTH=reg)
# vs the LDS-tiled AUTH pass: parity under the switch, then interleaved C2.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_vf2}; mkdir -p $O
NOISE_AEAD_VF_AUTH=reg timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_first.py tests/test_gpu_parity.py tests/test_config_digests.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "verify_first or VERIFY or duplex_solo_runs or full_size" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # tag env-assignment bench-args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -20 $O/$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),'seal',d['seal_gibs'],'open',d['open_gibs'])"
}
for rep in 1 2; do
  run c2_vf0_$rep X=1 --config c2
  run c2_vf1_lds_$rep X=1 --config c2 --verify-first
  run c2_vf1_reg_$rep NOISE_AEAD_VF_AUTH=reg --config c2 --verify-first
done
echo done

# Round 4: verify-first in one launch (one-lane ChaChaPoly AUTH + DEC passes,
# AES staged duplex) and the solo duplex's seal/open runs — parity, then
# interleaved C2 / C4 / C3 lines of both open orders (RUNS=0: block-by-block
# alternation, the previous placement).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_vf}; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_first.py tests/test_gpu_parity.py tests/test_config_digests.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "verify_first or duplex or full_size" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
fi
run() {  # tag env-assignment bench-args...
  local t=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { tail -20 $O/$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'),'seal',d['seal_gibs'],'open',d['open_gibs'])"
}
for rep in 1 2; do
  run c2_vf0_runs_$rep X=1 --config c2
  run c2_vf0_alt_$rep NOISE_AEAD_DUPLEX_RUNS=0 --config c2
  run c2_vf1_runs_$rep X=1 --config c2 --verify-first
  run c2_vf1_alt_$rep NOISE_AEAD_DUPLEX_RUNS=0 --config c2 --verify-first
  run c4_vf0_runs_$rep X=1 --config c4
  run c4_vf0_alt_$rep NOISE_AEAD_DUPLEX_RUNS=0 --config c4
  run c3_vf0_$rep X=1 --config c3
  run c3_vf1_$rep X=1 --config c3 --verify-first
done
echo done

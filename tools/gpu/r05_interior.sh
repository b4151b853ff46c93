# Round 5: seg ragged I/O interior-step fast path (NA_SEG_INTERIOR=1,
# default) against the per-instruction geometry (0): parity, cycle
# accounts, C5 interleaved.  Outputs in gpurun_out/r05_interior/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_interior}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_config_digests.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_seg.log 2>&1 || { tail -40 $O/pytest_seg.log; exit 1; }
tail -1 $O/pytest_seg.log
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_tl.so timeout -k 10 200 python tools/seg_tl.py > $O/tl.jsonl 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
cat $O/tl.jsonl
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));k=d.get('kernels_ms');print('$n',d['value'],d['ms_per_step'],d.get('verified'),k)"
}
for r in 1 2 3; do
b c5_int_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_noint.so b c5_noint_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

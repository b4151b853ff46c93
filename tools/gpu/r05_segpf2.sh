# Round 5: the next job's ticket + plan entries taken after the data pass
# (NA_SEG_PREFETCH=1, default) against at the top of the loop (0): parity,
# cycle accounts of both, C5 interleaved.  Outputs in gpurun_out/r05_segpf2/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r05_segpf2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py tests/test_config_digests.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_seg.log 2>&1 || { tail -40 $O/pytest_seg.log; exit 1; }
tail -1 $O/pytest_seg.log
for v in tl tlnopf; do
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$v.so timeout -k 10 200 python tools/seg_tl.py > $O/tl_$v.jsonl 2> $O/tl_$v.err || { tail -20 $O/tl_$v.err; exit 1; }
echo $v; cat $O/tl_$v.jsonl
done
b() {  # name bench-args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));k=d.get('kernels_ms');print('$n',d['value'],d['ms_per_step'],d.get('verified'),k)"
}
for r in 1 2 3; do
b c5_pf_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_nopf.so b c5_nopf_$r --config c5 --steps 20 --warmup 5 --no-cpu-baseline
done
echo done

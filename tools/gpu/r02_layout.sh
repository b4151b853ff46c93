# Open-side read amplification: 128-B slots (bench --align 128) and
# non-temporal record stores (variant "nt") vs the default, C2/C4 speed
# interleaved, then FETCH/WRITE passes for each.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_layout; mkdir -p $O
run() { # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$lib.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 8 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],'seal',d['seal_gibs'],'open',d['open_gibs'])"
}
for i in 1 2; do
  for c in c2 c4; do
    run $c.cur.$i cur --config $c
    run $c.a128.$i cur --config $c --align 128
    run $c.nt.$i nt --config $c
  done
done
cd /tmp && export TMPDIR=/tmp
pmc() { # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$lib.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_$tag/$ctr -o run --output-format csv -- python3 $R/bench.py --config c2 --no-cpu-baseline --steps 10 --warmup 2 "$@" > $O/pmc_$tag.$ctr.log 2>&1 || { echo "pmc $tag $ctr failed"; tail -5 $O/pmc_$tag.$ctr.log; exit 1; }
  done
  python3 $R/tools/pmc_report.py $O/pmc_$tag c2 $O/traffic_$tag.json | grep -E "chacha" | cut -c1-200
}
pmc a128 cur --align 128
pmc nt nt
echo layout done

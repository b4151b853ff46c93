# Round 5: the verify-first AUTH pass at the default priority
# (-DNA_SOLO_NO_AUTH_PRIO, ab/libnoise_aead_hip_noprio.so) vs s_setprio 3,
# two steps in flight either way: C2 --verify-first interleaved.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_vfprio; mkdir -p $O
X=$R/noise-c_amd/ab/libnoise_aead_hip_noprio.so
b() { local n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('verified'))"; }
for r in 1 2 3; do
b prio3_$r python bench.py --config c2 --verify-first --steps 20 --warmup 5 --no-cpu-baseline
NOISE_AEAD_LIB=$X b noprio_$r python bench.py --config c2 --verify-first --steps 20 --warmup 5 --no-cpu-baseline
done

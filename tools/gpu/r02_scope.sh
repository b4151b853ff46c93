# Store cache policy of the staged ChaChaPoly kernels' record stores:
# cur (plain global stores) vs sc1 / sc0+sc1 buffer stores (variants),
# C2/C4 interleaved with --verify, then per variant a kernel trace of C2
# (duplex durations and the gaps between launches) and WRITE_SIZE.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_scope; mkdir -p $O
V=${VARIANTS:-sc1 sc01}
use() { if [ "$1" = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$1.so; fi; }
for i in 1 2; do
  for v in cur $V; do
    use $v
    for c in c2 c4; do
      timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 8 --verify > $O/$c.$v.$i.json 2> $O/$c.$v.$i.err || { tail -20 $O/$c.$v.$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$c.$v.$i.json'));print('$c $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],'seal',d['seal_gibs'],'open',d['open_gibs'],d.get('verified'))"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for v in cur $V; do
  use $v
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_$v -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $O/kt_$v.log 2>&1 || { tail -20 $O/kt_$v.log; exit 1; }
  (cd $R && python3 tools/kgaps.py $O/kt_$v chachapoly_duplex) | sed "s/^/$v /"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pw_$v -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/pw_$v.log 2>&1 || { tail -5 $O/pw_$v.log; exit 1; }
  (cd $R && python3 tools/pmc_report.py $O/pw_$v c2 $O/tr_$v.json | grep duplex | cut -c1-120 | sed "s/^/$v /")
done
echo scope done

# rocprofv3 kernel stats of the C5 bench (final kernels).
set -u
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5f -o run --output-format csv -- python3 $R/bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 > $R/gpurun_out/prof_c5f.log 2>&1 || { tail -20 $R/gpurun_out/prof_c5f.log; exit 1; }
echo prof done

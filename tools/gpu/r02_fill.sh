# C5 HBM-traffic passes on the final kernels, and the C3 line with its
# AES-GCM CPU reference baseline.
set -u
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r02_fill; mkdir -p $O
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3_cpu.json 2> $O/bench_c3_cpu.err || { tail -20 $O/bench_c3_cpu.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3_cpu.json'));print(d['value'],d['cpu_baseline'])"
bash tools/gpu/traffic.sh c5 || exit 1
cp $R/gpurun_out/traffic_c5.json $O/
echo fill done

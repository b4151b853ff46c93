# Round 4: PMC passes (FETCH/WRITE/SQ/busy/TCC) of every bench config's step
# kernel on the final code -> gpurun_out/traffic_<cfg>.json (copied into
# profiles/ for bench.py's roofline.traffic and issue_bound).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/traffic.sh ${CFGS:-c2 c3 c4 perf c5}

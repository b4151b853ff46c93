# HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, TCC) for the named configs,
# summarised into gpurun_out/traffic_<cfg>.json (copied into profiles/ by hand).
set -eu
R=$GRAFT_REPO_ROOT; cd $R
for cfg in "$@"; do
  bash tools/gpu/pmc.sh $cfg $R/gpurun_out/pmc_$cfg
  python3 tools/pmc_report.py $R/gpurun_out/pmc_$cfg $cfg $R/gpurun_out/traffic_$cfg.json > /dev/null
done
echo traffic done

# Round 4: PMC passes (instruction counts, wave/busy cycles, HBM bytes) of
# the duplex kernels at 1 and 4 lanes per record, C2 and C4.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${ROUND_DIR:-r04_pmc}; mkdir -p $O
for cfg in ${CFGS:-c2 c4}; do
  for k in ${LANES:-4 1}; do
    PMC_GROUPS="${PMC_GROUPS:-fetch write sq busy}" bash tools/gpu/pmc.sh $cfg $O/pmc_${cfg}_k$k --lanes $k
    python3 tools/pmc_report.py $O/pmc_${cfg}_k$k $cfg $O/traffic_${cfg}_k$k.json | grep -v copyBuffer | cut -c1-900
  done
done
echo done

# Round 5: LDS counters of the AES-GCM kernels (C3 fused duplex, C5 ragged
# seal/open, one stream) and of C5's ChaChaPoly seg kernels, plus the
# instruction counts.  Outputs in gpurun_out/r05_pmc_lds/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_pmc_lds; mkdir -p $O
PMC_GROUPS="lds busy" bash tools/gpu/pmc.sh c3 $O/c3
PMC_GROUPS="lds busy" bash tools/gpu/pmc.sh c5 $O/c5 --c5-streams 1
python3 - <<'PY'
import csv, glob, os, collections
O=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/r05_pmc_lds'
for run in ('c3','c5'):
    agg=collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f'{O}/{run}/*/**/*counter_collection.csv', recursive=True):
        for row in csv.DictReader(open(f)):
            agg[row['Kernel_Name'][:70]][row['Counter_Name']].append(float(row['Counter_Value']))
    for k,v in agg.items():
        if 'gcm' not in k and 'chacha' not in k: continue
        print(run, k, {c: round(sum(x)/len(x)) for c,x in v.items()})
PY

# PMC (SQ instruction and busy counters) of the segmented kernels against
# the one-lane duplex: the standalone C2 seal/open (--mode separate: the
# seg2 kernels), C5 (the planned ragged kernels), C2 duplex.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_pmc_seg; mkdir -p $O
PMC_GROUPS="sq busy" bash tools/gpu/pmc.sh c2 $O/sep --mode separate
PMC_GROUPS="sq busy" bash tools/gpu/pmc.sh c2 $O/dup
PMC_GROUPS="sq busy" bash tools/gpu/pmc.sh c5 $O/c5 --c5-streams 1
python3 - <<'PY'
import csv, glob, os, collections
O=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/r05_pmc_seg'
for run in ('sep','dup','c5'):
    agg=collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f'{O}/{run}/*/**/*counter_collection.csv', recursive=True):
        for row in csv.DictReader(open(f)):
            agg[row['Kernel_Name'][:60]][row['Counter_Name']].append(float(row['Counter_Value']))
    for k,v in agg.items():
        if 'chacha' not in k: continue
        print(run, k, {c: round(sum(x)/len(x)) for c,x in v.items()})
PY

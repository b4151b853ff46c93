# PMC passes for the bench kernels (one rocprofv3 run per counter group;
# --pmc with --kernel-trace only, as the pool requires).  Usage:
#   bash tools/gpu/pmc.sh CONFIG OUTDIR [extra bench args]
set -u
R=$GRAFT_REPO_ROOT
CFG=${1:-c2}; OUT=${2:-$R/gpurun_out/pmc_$CFG}; shift 2 || true
EXTRA="$@"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
      python3 $R/bench.py --config $CFG --no-cpu-baseline --no-verify --settle-ms 0 --steps 10 --warmup 2 $EXTRA > $OUT/$name.log 2>&1
  echo "pmc $name rc=$?"
}
# PMC_GROUPS: a subset of the passes (default all five)
G=" ${PMC_GROUPS:-fetch write sq busy tcc} "
case "$G" in *" fetch "*) run fetch FETCH_SIZE || exit 1;; esac
case "$G" in *" write "*) run write WRITE_SIZE || exit 1;; esac
case "$G" in *" sq "*) run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1;; esac
case "$G" in *" busy "*) run busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY || exit 1;; esac
case "$G" in *" tcc "*) run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum || exit 1;; esac
# LDS: array cycles, bank-conflict cycles, issue stalls (opt-in: PMC_GROUPS="lds")
case "$G" in *" lds "*) run lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1;; esac

# Instruction-mix / issue PMC passes only (see pmc.sh).  Usage: bash tools/gpu/pmc_sq.sh CONFIG [bench args]
set -u
R=$GRAFT_REPO_ROOT
CFG=${1:-c2}; shift || true
OUT=$R/gpurun_out/pmcsq_$CFG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
      python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 10 --warmup 2 "$EXTRA_ARGS" > $OUT/$name.log 2>&1
  echo "pmc $name rc=$?"
}
EXTRA_ARGS="${*:---sets=4}"
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1
run busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY || exit 1
run lds SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS || exit 1

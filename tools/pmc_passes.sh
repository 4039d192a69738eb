#!/bin/bash
# Collect rocprofv3 PMC counters for the MMSE kernels, one pass per counter
# group (counters never combined with sys/runtime traces).  Output under
# gpurun_out/pmc/<pass>/.  Usage: tools/pmc_passes.sh [bench args...]
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${PMC_DIR:-pmc}
mkdir -p "$OUT"
# PMC_EXTRAS=1: profile every bench leg (LS, front end, config 5, ...), not just the headline
EXTRAS=--no-extras
[ -n "$PMC_EXTRAS" ] && EXTRAS=
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" \
     -- python3 "$ROOT/bench.py" $EXTRAS --steps 5 --no-cpu-baseline --warmup 1 ${BENCH_ARGS} \
     > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 &&
run grbm GRBM_GUI_ACTIVE GRBM_COUNT &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run mfma SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64
echo "pmc passes done: $?"

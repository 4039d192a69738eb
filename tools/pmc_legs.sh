#!/bin/bash
# rocprofv3 PMC passes over each bench leg's dominant kernel ALONE, at the
# bench's launch size (tools/prof_leg.py), one pass per counter group (never
# combined with sys/runtime traces; each pass within the per-block limits).
# -> gpurun_out/pmc_legs/<leg>/<pass>/ and, summarised per dispatch,
#    gpurun_out/pmc_legs.json (copy to profiles/<round>_pmc_legs.json).
# usage: tools/pmc_legs.sh [leg ...]   (default: every leg)
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_legs
mkdir -p "$OUT"
LEGS=${*:-"headline apply apply1m cov_solve ref ls ls_pilots front_blocks front_preamble config5 config5_ref config5_ref_f32 lowrank4 lowrank8 lowrank16 lowrank24 lowrank53 lowrank8_1m config5_ref_fc config5_ref_fc_factors frame_cov_ref cm16 cm53"}
run() {
  local leg=$1 name=$2; shift 2
  mkdir -p "$OUT/$leg"
  timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$leg/$name" -o run --pmc "$@" \
     -- python3 "$ROOT/tools/prof_leg.py" --leg "$leg" --reps 5 > "$OUT/$leg/$name.log" 2>&1
}
for leg in $LEGS; do
  run $leg sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
  run $leg grbm GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
  run $leg fetch FETCH_SIZE || exit $?
  run $leg write WRITE_SIZE || exit $?
  case $leg in
    headline|cov_solve|apply|apply1m|config5|lowrank*|cm*|frame_cov_ref)
      run $leg sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 || exit $? ;;
  esac
  if [ "$leg" = apply ] || [ "$leg" = apply1m ] || [ "${leg#lowrank}" != "$leg" ] || [ "${leg#cm}" != "$leg" ] || [ "$leg" = frame_cov_ref ]; then
    run $leg mfma SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 || exit $?
  fi
  echo "leg $leg done"
done
python3 "$ROOT/tools/pmc_legs_summary.py" "$OUT" "$ROOT/gpurun_out/pmc_legs.json" && echo "pmc legs done"

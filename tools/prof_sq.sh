#!/bin/bash
# SQ/TA counter passes (one rocprofv3 run per pass, kernel trace only) on one
# bench configuration. usage: bash tools/prof_sq.sh <outdir> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
run() {
  local name=$1; local ctrs=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/$name -o run \
    -- python3 bench.py "$@" --cpu-sample 0 --no-verify > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "$@"
run sq2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "$@"
run ta "TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum" "$@"

#!/bin/bash
# Per-kernel rocprofv3 counter passes on one bench configuration.
# usage: bash tools/prof_counters.sh <outdir> [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
ARGS="$@"
mkdir -p $OUT
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python bench.py $ARGS --cpu-sample 0 --no-verify > $OUT/$name.log 2>&1
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py $ARGS --cpu-sample 0 --no-verify > $OUT/trace.log 2>&1
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum
run utcl TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
echo done

#!/bin/bash
# Round profile of the headline bench command (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of `python bench.py <args>`
#   2. a FETCH_SIZE pass and a WRITE_SIZE pass (separate: they do not fit one
#      pass on gfx950), kernel trace only, no runtime/sys traces
# Outputs under gpurun_out/prof/<tag>/; tools/profile_summary.py turns them
# into profiles/<tag>_*.{csv,json,md}.
# usage: bash tools/profile_round.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 bench.py "$@" > $OUT/bench_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run \
  -- python3 bench.py "$@" --cpu-sample 0 > $OUT/bench_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
echo "fetch ok"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run \
  -- python3 bench.py "$@" --cpu-sample 0 > $OUT/bench_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo "write ok"

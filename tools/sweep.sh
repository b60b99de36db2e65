#!/bin/bash
# Bench every built variant (simd-radix-sort_amd/lib/variants/*) at one size.
# usage: tools/sweep.sh <n> [variant ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=$1; shift
VARS="$@"; [ -z "$VARS" ] && VARS=$(ls simd-radix-sort_amd/lib/variants)
mkdir -p gpurun_out/sweep
for v in $VARS; do
  SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so timeout -k 10 300 \
    python bench.py --n $N --config ${CFG:-c1} --steps 3 --cpu-sample 0 > gpurun_out/sweep/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/sweep/$v.log | cut -c1-120)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done

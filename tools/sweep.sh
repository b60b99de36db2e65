#!/bin/bash
# Bench built variants (simd-radix-sort_amd/lib/variants/*) at one size, in the
# order given (repeat names to interleave A/B runs on the same box).
# usage: [CFG=c2] tools/sweep.sh <n> variant ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=$1; shift
VARS="$@"; [ -z "$VARS" ] && VARS=$(ls simd-radix-sort_amd/lib/variants)
mkdir -p gpurun_out/sweep
i=0
for v in $VARS; do
  i=$((i+1))
  log=gpurun_out/sweep/${CFG:-c1}_${i}_$v.log
  SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so timeout -k 10 300 \
    python bench.py --n $N --config ${CFG:-c1} --steps ${STEPS:-3} --cpu-sample 0 > $log 2>&1
  rc=$?
  echo "$v rc=$rc $(python tools/show.py $log | cut -d' ' -f2-)" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done

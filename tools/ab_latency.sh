#!/bin/bash
# Interleaved latency A/B of library builds: tools/latency.py at the given
# sizes for each variant in $VARS ("cur" = the in-tree library, else
# simd-radix-sort_amd/lib/variants/<v>/), $REPS rounds.
# usage: VARS="cur sg64" bash tools/ab_latency.sh <out> n [n ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:?usage: ab_latency.sh <out> n...}; shift
mkdir -p "$OUT"
for i in $(seq ${REPS:-2}); do for v in $VARS; do
  if [ $v = cur ]; then lib=$PWD/simd-radix-sort_amd/lib/libsrs_amd.so
  else lib=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so; fi
  SRS_AMD_LIB=$lib timeout -k 10 120 python tools/latency.py "$@" > "$OUT/${v}_$i.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "$OUT/${v}_$i.log"; exit $rc; }
  grep "n=" "$OUT/${v}_$i.log" | sed "s/^/$v $i /"
done; done

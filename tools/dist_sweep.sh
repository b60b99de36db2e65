#!/bin/bash
# C1 (u64 key + u64 payload, 1e9) over the reference's eight input
# distributions (src/data.hpp:64-97), one bench process each (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/dist
for d in uniform gaussian zero zeroone sorted reverse almostsorted almostreverse; do
  SRS_TRACE_LEVELS=${TRACE:-0} timeout -k 10 300 python bench.py --dist $d --steps ${STEPS:-3} --cpu-sample 0 --extra none \
    > gpurun_out/dist/$d.log 2>&1; rc=$?
  echo "$d rc=$rc $(python tools/show.py gpurun_out/dist/$d.log | cut -d' ' -f2-4)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

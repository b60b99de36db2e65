#!/bin/bash
# Kernel-trace each variant library (lib/variants/<v>) on one bench config:
# per-dispatch durations land in gpurun_out/kt/<v>/ (tools/kt_table.py reads them).
# usage: VARS="base cur" CFG=c1 bash tools/kt_variants.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/kt; export TMPDIR=/tmp
for v in $VARS; do
  rm -rf gpurun_out/kt/$v
  SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so timeout -k 10 300 \
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt/$v -o kt -- \
    python bench.py --config ${CFG:-c1} --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 --no-verify $EXTRA \
    > gpurun_out/kt/$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done; exit 0

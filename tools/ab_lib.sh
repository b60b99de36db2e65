#!/bin/bash
# Interleaved A/B of library builds on the bench: for each config in $CFGS,
# runs each variant in $VARS (simd-radix-sort_amd/lib/variants/<v>/, "cur" =
# the in-tree library) $REPS times; one summary line per run.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ablib
for c in ${CFGS:-c1}; do for i in $(seq ${REPS:-2}); do for v in $VARS; do
  log=gpurun_out/ablib/${c}_${v}_$i.log
  if [ $v = cur ]; then lib=$PWD/simd-radix-sort_amd/lib/libsrs_amd.so
  else lib=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so; fi
  SRS_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --cpu-sample 0 --extra none $EXTRA > $log 2>&1
  rc=$?; echo "$c $v rc=$rc $(python tools/show.py $log | cut -d' ' -f2-)" | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done; done; done; exit 0

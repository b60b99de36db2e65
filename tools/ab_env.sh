#!/bin/bash
# Interleaved A/B of one environment switch on the bench: for each config in
# $CFGS, runs "$OFF" (env assignment, e.g. SRS_NO_STRIPES=1) then the default,
# $REPS times; prints one summary line per run.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abenv
for c in ${CFGS:-c1}; do for i in $(seq ${REPS:-2}); do for v in off on; do
  log=gpurun_out/abenv/${c}_${v}_$i.log
  if [ $v = off ]; then env $OFF timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --cpu-sample 0 > $log 2>&1
  else timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --cpu-sample 0 > $log 2>&1; fi
  rc=$?; echo "$c $v rc=$rc $(python tools/show.py $log | cut -d' ' -f2-)" | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done; done; done; exit 0

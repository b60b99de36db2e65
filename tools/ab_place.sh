#!/bin/bash
# A/B of the placement-probed allocation, interleaved on one
# box: arm "placed" = defaults (workspace and outputs probed and re-placed),
# arm "plain" = SRS_PLACE=0 and torch-allocated outputs (round 3's setup).
# N fresh bench processes per arm (C1 only), one summary line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/abp
N=${N:-5}
for i in $(seq 1 $N); do
  for arm in placed plain; do
    log=gpurun_out/abp/${arm}_$i.log
    if [ $arm = plain ]; then
      SRS_PLACE=0 timeout -k 10 300 python bench.py --steps ${STEPS:-10} --cpu-sample 0 --extra none --out-alloc torch > $log 2>&1
    else
      timeout -k 10 300 python bench.py --steps ${STEPS:-10} --cpu-sample 0 --extra none > $log 2>&1
    fi
    rc=$?
    [ $rc -ne 0 ] && { echo "$arm $i rc=$rc"; tail -5 $log; exit $rc; }
    python - "$log" "$arm" "$i" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["kernels"]
g = lambda n: k.get(n, {}).get("avg_ms")
print(f"{sys.argv[2]:6s} {sys.argv[3]} ms/step {d['ms_per_step']:.3f} plain {d['ms_per_step_without_event_markers']:.3f} "
      f"scatter.L1 {g('scatter.L1')} scatter.L2 {g('scatter.L2')} local {g('local')} count {g('count')} "
      f"verified {all(d['verified'].values())}", flush=True)
PY
  done
done

#!/bin/bash
# Interleaved A/B of library variants (lib/variants/<name>/libsrs_amd.so) on
# bench configs, printing ms/step and the per-level kernel times.
# usage: VARS="base x" CFGS="c2 c1" REPS=2 bash tools/ab_levels.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in $(seq ${REPS:-2}); do for c in ${CFGS:-c2}; do for v in $VARS; do
  log=gpurun_out/ab/${c}_${v}_$r.json
  SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so timeout -k 10 200 \
    python bench.py --config $c --steps ${STEPS:-10} --extra none --cpu-sample 0 $EXTRA > $log 2> ${log%.json}.err
  rc=$?; [ $rc -ne 0 ] && { echo "$c $v rc=$rc"; tail -3 ${log%.json}.err; exit $rc; }
  python3 - "$log" "$c" "$v" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
k = d["kernels"]
lv = " ".join(f"{n}={v['avg_ms']:.3f}" for n, v in k.items() if ".L" in n or n in ("local", "scan"))
print(f"{sys.argv[2]} {sys.argv[3]:8s} {d['ms_per_step']:.3f} ms  {lv}")
PY
done; done; done

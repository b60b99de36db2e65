#!/bin/bash
# One parameterised GPU session (replaces the single-use round-5 wrappers):
#   bash tools/gpu_run.sh <out> step [step ...]
# Steps (each under its own time limit, output in gpurun_out/<out>/<name>.log):
#   smoke        __graft_entry__ smoke
#   tests        the whole -m gpu suite
#   t:<expr>     -m gpu tests selected by -k <expr>  (e.g. t:shard)
#   f:<file>     -m gpu tests of tests/<file>.py
#   exitcheck    the mid-size sorts under rocprofv3 --kernel-trace (the exit-time
#                crash of VERDICT r05), exit status recorded
#   b9 / c2 / c3 bench.py at 1e9 (3 steps, no CPU baseline) for C1 / C2 / C3
#   shard        bench.py --shard (world 1, RCCL, 8 chunks / 16 rounds)
#   shardself    the same with self messages (own pieces through ncclSend/Recv)
#   shardspan8   the same over keys confined to 1/8 of the key range (one of 8 ranks' span)
#   profiles     tools/round_profiles.sh $PROFILE_TAG (C1 / C2 / C3 traces + PMC passes)
#   lat          tools/latency.py over the small / mid sizes
#   latab        tools/latency.py at 1M-4M keys without / with the mid-level launch
#   phases       tools/latency_phases.py (kernel time per family), without / with the mid-level launch
#   bench        the default bench.py line (what the driver runs)
# After a crash, abort or time limit (rc >= 124, 134, 139) nothing else runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:?usage: gpu_run.sh <out> step...}
shift
mkdir -p "$OUT"
: > "$OUT/steps.txt"
export TMPDIR=/tmp
LATN="1048577 1500000 2097152 3000000 3900000 4194304 6000000"
PT="python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/steps.txt"
  tail -3 "$OUT/$name.log" | sed "s/^/[$name] /"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "STOP after $name rc=$rc"; cat "$OUT/steps.txt"; exit $rc
  fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    tests) step pytest_gpu 900 $PT tests ;;
    t:*) step "pytest_${s#t:}" 600 $PT tests -k "${s#t:}" ;;
    f:*) step "pytest_${s#f:}" 600 $PT "tests/${s#f:}.py" ;;
    exitcheck) step exitcheck 300 rocprofv3 --kernel-trace -d "$OUT/exitcheck_prof" -o run -- \
                 python tools/latency.py 8192 8193 32768 262144 ;;
    b9) step bench_c1 600 python bench.py --steps 3 --cpu-sample 0 --extra none ;;
    c2) step bench_c2 600 python bench.py --config c2 --steps 3 --cpu-sample 0 --extra none ;;
    c3) step bench_c3 600 python bench.py --config c3 --steps 3 --cpu-sample 0 --extra none ;;
    shard) step bench_shard 600 python bench.py --shard --steps 3 --cpu-sample 0 ;;
    shardself) step bench_shard_self 600 python bench.py --shard --self-messages --steps 3 \
                 --cpu-sample 0 ;;
    shardspan8) step bench_shard_span8 600 python bench.py --shard --dist span8 --steps 3 \
                 --cpu-sample 0 ;;
    profiles) step profiles 1500 bash tools/round_profiles.sh "${PROFILE_TAG:-r06}" ;;
    lat) step latency 300 python tools/latency.py ;;
    latab) step latency_general 300 env SRS_MID_LEVEL_MAX=0 python tools/latency.py $LATN &&
           step latency_midlevel 300 python tools/latency.py $LATN ;;
    phases) step phases_general 300 env SRS_MID_LEVEL_MAX=0 python tools/latency_phases.py $LATN &&
            step phases_midlevel 300 python tools/latency_phases.py $LATN ;;
    bench) step bench_default 900 python bench.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
cat "$OUT/steps.txt"

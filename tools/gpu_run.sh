#!/bin/bash
# Standard GPU session: smoke, GPU tests, benches. Each GPU step has its own
# time limit; after a crash/abort/timeout (rc >= 124 or rc 134/139) nothing
# else touches the GPU. A plain test failure (rc 1) does not stop the benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/steps.txt
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name rc=$rc"; exit $rc; fi
  return 0
}
: > gpurun_out/steps.txt
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    b8) step bench_1e8 300 python bench.py --n 1e8 --steps 3 --cpu-sample 0 ;;
    b9) step bench_1e9 600 python bench.py --steps 3 --cpu-sample 0 ;;
    b9full) step bench_1e9_full 900 python bench.py ;;
    c2) step bench_c2 600 python bench.py --config c2 --steps 3 --cpu-sample 0 ;;
    c3) step bench_c3 600 python bench.py --config c3 --steps 3 --cpu-sample 0 ;;
    shard) step bench_shard 600 python bench.py --shard --steps 3 --cpu-sample 0 ;;
    shardc2) step bench_shard_c2 600 python bench.py --shard --config c2 --steps 3 --cpu-sample 0 ;;
  esac
done
cat gpurun_out/steps.txt

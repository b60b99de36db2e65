#!/bin/bash
# GPU session: new tests first, then the full -m gpu suite, then the default bench line.
# usage: bash tools/gpu_quick.sh [pytest selection...]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/steps.txt
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -ne 0 ] && { tail -30 gpurun_out/$n.log; exit $rc; }; return 0; }
st pytest_sel 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu ${SEL:-tests/test_gpu_ref_full.py tests/test_bench.py tests/test_cpp_dropin.py}
tail -3 gpurun_out/pytest_sel.log
[ -n "$FULL" ] && { st pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread; tail -2 gpurun_out/pytest_gpu.log; }
st bench 500 python bench.py
tail -c 3000 gpurun_out/bench.log

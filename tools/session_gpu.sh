#!/bin/bash
# One GPU session: smoke, the -m gpu suite, the three round profiles
# (tools/round_profiles.sh <tag>) and the default bench line.
# usage: bash tools/session_gpu.sh <tag>
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/steps.txt
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -ne 0 ] && { tail -30 gpurun_out/$n.log; exit $rc; }; return 0; }
st smoke 300 python __graft_entry__.py smoke
st pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
bash tools/round_profiles.sh $1 || exit 1
st bench 500 python bench.py
python tools/show.py gpurun_out/bench.log | cut -c1-400

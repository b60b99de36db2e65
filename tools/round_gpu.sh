#!/bin/bash
# Round-end GPU session: smoke, GPU tests, round profile (tools/profile_round.sh <tag>), C2/C3 benches.
# usage: bash tools/round_gpu.sh <tag>
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/steps.txt
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -ge 124 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc; return 0; }
st smoke 300 python __graft_entry__.py smoke
st pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
TAG=${1:-r02}
bash tools/profile_round.sh $TAG || exit 1
st bench_c2 400 python bench.py --config c2 --steps 3 --cpu-sample 0
st bench_c3 400 python bench.py --config c3 --steps 3 --cpu-sample 0
for f in gpurun_out/prof/$TAG/bench_trace.log gpurun_out/bench_c2.log gpurun_out/bench_c3.log; do python tools/show.py $f | cut -c1-330; done
st perf_dat 900 python tools/perf_dat.py --out gpurun_out/perf_dat

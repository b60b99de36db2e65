#!/bin/bash
# Where a shard round sort's time goes (world 1, RCCL): plain sorts of one
# round's size next to 1e9 (tools/latency.py, latency_phases.py), then a
# rocprofv3 kernel trace of `bench.py --shard`, summarised per kernel.
# usage: bash tools/prof_rounds.sh <outdir under gpurun_out>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rounds}
mkdir -p $OUT
export TMPDIR=/tmp
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.txt 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$n.txt; exit $rc; }; return 0; }
st latency 300 python tools/latency.py 16777216 33554432 67108864 125000000 134217728
st phases 300 python tools/latency_phases.py 16777216 125000000 134217728
st shard_trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o shard -- \
  python bench.py --shard --steps 2 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0
tail -3 $OUT/latency.txt
# outputs the library did not place: per-kernel times of the in-place arm
st ab_outputs 400 python tools/ab_outputs.py --sets placed,inplace,plain,placed,inplace --rounds 5
st ab_outputs_nohome 400 env SRS_HOME_TMP2=0 python tools/ab_outputs.py --sets placed,inplace,plain --rounds 5

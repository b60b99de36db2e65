#!/bin/bash
# Full GPU check of a library change: the -m gpu suite, a kernel trace of the
# world-1 shard line, the shard line with and without the super-group scan
# (interleaved), then the default bench line.
# usage: bash tools/session_final.sh <outdir under gpurun_out>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
export TMPDIR=/tmp
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.txt 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$n.txt; exit $rc; }; return 0; }
st smoke 300 python __graft_entry__.py smoke
st pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $OUT/pytest_gpu.txt
st shard_trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o shard -- \
  python bench.py --shard --steps 2 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0
B="python bench.py --shard --steps 5 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0"
st shard_a1 300 $B
st shard_b1 300 env SRS_SUPER_SCAN=0 $B
st shard_a2 300 $B
st shard_b2 300 env SRS_SUPER_SCAN=0 $B
st bench 500 python bench.py
for f in shard_a1 shard_b1 shard_a2 shard_b2 bench; do python tools/show.py $OUT/$f.txt | cut -c1-160; done

#!/bin/bash
# Shard-path check after a library change: the shard and sort GPU tests, a
# kernel trace of `bench.py --shard` (world 1), then the shard line with and
# without the partition's tile-pair scatter, interleaved.
# usage: bash tools/shard_ab.sh <outdir under gpurun_out>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-shard_ab}
mkdir -p $OUT
export TMPDIR=/tmp
st() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.txt 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$n.txt; exit $rc; }; return 0; }
st tests 600 python -u -m pytest tests/test_shard_gpu.py tests/test_gpu_sort.py -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $OUT/tests.txt
st shard_trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o shard -- \
  python bench.py --shard --steps 2 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0
B="python bench.py --shard --steps 5 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0"
st shard_a1 300 $B
st shard_b1 300 env SRS_PARTITION_PAIRS=0 $B
st shard_a2 300 $B
st shard_b2 300 env SRS_PARTITION_PAIRS=0 $B
for f in a1 b1 a2 b2; do python tools/show.py $OUT/shard_$f.txt | cut -c1-160; done

#!/bin/bash
# SQ counters of the count kernel: the product's (bench C2) against the
# probe's (tools/probe/count_probe). usage: bash tools/prof_count.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/bench$i -o run \
    -- python3 bench.py --config c2 --steps 2 --warmup 1 --extra none --cpu-sample 0 --no-verify \
    > $OUT/bench$i.log 2>&1 || { echo "bench pass $i rc=$?"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/probe$i -o run \
    -- ./tools/probe/count_probe > $OUT/probe$i.log 2>&1 || { echo "probe pass $i rc=$?"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py $(find $OUT/bench1 $OUT/bench2 -name "*counter_collection.csv") | grep count_kernel > $OUT/bench_count.txt
python3 tools/pmc_summary.py $(find $OUT/probe1 $OUT/probe2 -name "*counter_collection.csv") | grep count_kernel > $OUT/probe_count.txt
cat $OUT/bench_count.txt $OUT/probe_count.txt | cut -c1-1500

# round 5, GPU call l: the whole GPU suite, then two default bench lines (no CPU baselines)
set -o pipefail
mkdir -p gpurun_out/r5l
T="timeout -k 10"
$T 700 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5l/t.txt 2>&1 || exit 1
for i in 1 2; do
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5l/b$i.json 2> gpurun_out/r5l/b$i.err || exit 2
done

# round 5, GPU call i: shard tests after the schedule change, placement, bench lines,
# shard world-1 head/tail at several rounds/chunks
set -o pipefail
mkdir -p gpurun_out/r5i
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_shard_gpu.py tests/test_cpp_dropin.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5i/t.txt 2>&1 || exit 1
$T 300 python -u tools/ab_outputs.py --sets placed,plain,placed,plain > gpurun_out/r5i/ab.json 2> gpurun_out/r5i/ab.err || exit 2
for i in 1 2; do
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5i/b$i.json 2> gpurun_out/r5i/b$i.err || exit 3
done
for rc in "8 1" "16 8" "8 8" "16 16"; do
  set -- $rc
  $T 300 python -u bench.py --shard --steps 5 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0 --rounds $1 --chunks $2 > gpurun_out/r5i/shard_r$1_c$2.json 2> gpurun_out/r5i/shard_r$1_c$2.err || exit 4
done

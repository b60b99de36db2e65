# round 5, GPU call n: mid-size parity, then kernel durations of small /
# mid-size calls (kernel trace) and plain per-call latency
set -o pipefail
mkdir -p gpurun_out/r5n
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_mid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n/mid_t.txt 2>&1 || exit 1
$T 200 python -u tools/latency.py 4096 8192 8193 16384 32768 65536 131072 262144 524288 > gpurun_out/r5n/lat.txt 2>&1 || exit 2
$T 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5n/mid -o run -- python tools/latency.py 8193 32768 262144 > gpurun_out/r5n/mid.txt 2>&1 || exit 3

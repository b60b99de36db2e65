# round 5, GPU call m: the mid-size single launch -- its parity tests, the
# size sweep of test_gpu_sort, then per-call latency with and without it
set -o pipefail
mkdir -p gpurun_out/r5m
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_mid.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5m/mid.txt 2>&1 || exit 1
$T 400 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 200 --timeout-method thread -k "sizes or distributions or fallback" > gpurun_out/r5m/sort.txt 2>&1 || exit 2
$T 200 python -u tools/latency.py 4096 8192 8193 16384 32768 65536 131072 262144 524288 > gpurun_out/r5m/lat_mid.txt 2>&1 || exit 3
SRS_MID=0 $T 200 python -u tools/latency.py 8193 16384 32768 65536 131072 262144 > gpurun_out/r5m/lat_nomid.txt 2>&1 || exit 4

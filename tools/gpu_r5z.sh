# round 5, GPU call z: the mid-size launch with its own grid barrier
set -o pipefail
mkdir -p gpurun_out/r5z
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_mid.py -x -q --timeout 60 --timeout-method thread > gpurun_out/r5z/mid.txt 2>&1 || exit 1
$T 600 python -u -m pytest tests/test_gpu_sort.py tests/test_capi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5z/t.txt 2>&1 || exit 2
$T 200 python -u tools/latency.py 8192 8193 16384 32768 65536 131072 262144 > gpurun_out/r5z/lat.txt 2>&1 || exit 3
$T 120 ./tools/probe/grid_sync > gpurun_out/r5z/grid_sync.txt 2>&1 || exit 4

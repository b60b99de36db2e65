# round 5, GPU call w: small sorts with 12 / 13-bit bucket digits
set -o pipefail
mkdir -p gpurun_out/r5w
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_mid.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5w/t.txt 2>&1 || exit 1
$T 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5w/sp -o run -- python tools/small_paths.py > gpurun_out/r5w/sp.txt 2>&1 || exit 2
$T 200 python -u tools/latency.py 16 256 1024 2048 4096 8192 8193 65536 262144 > gpurun_out/r5w/lat.txt 2>&1 || exit 3

# round 5, GPU call u: DPP / ballot wave reductions -- parity of the local
# bodies, small-sort stamps and kernel times
set -o pipefail
mkdir -p gpurun_out/r5u
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_mid.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5u/t.txt 2>&1 || exit 1
SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/stamps/libsrs_amd.so $T 120 python tools/stamps_small.py 1024 4096 > gpurun_out/r5u/stamps.txt 2>&1 || exit 2
$T 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5u/sp -o run -- python tools/small_paths.py > gpurun_out/r5u/sp.txt 2>&1 || exit 3
SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/twice/libsrs_amd.so $T 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5u/twice -o run -- python tools/small_paths.py > gpurun_out/r5u/twice.txt 2>&1 || exit 4

# round 5, GPU call t: wave-reduced LDS max/or -- small-sort stamps and
# kernel times, then the default line with the previous and the new library
set -o pipefail
mkdir -p gpurun_out/r5t
T="timeout -k 10"
SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/stamps/libsrs_amd.so $T 120 python tools/stamps_small.py 1024 4096 > gpurun_out/r5t/stamps.txt 2>&1 || exit 1
$T 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5t/sp -o run -- python tools/small_paths.py > gpurun_out/r5t/sp.txt 2>&1 || exit 2
for i in 1 2; do
  SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/base/libsrs_amd.so $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5t/base$i.json 2> gpurun_out/r5t/base$i.err || exit 3
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5t/new$i.json 2> gpurun_out/r5t/new$i.err || exit 4
done

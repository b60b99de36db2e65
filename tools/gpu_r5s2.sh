# round 5: polled control read-backs -- the previous library (variants/base2)
# and the new one, alternated, default line without CPU baselines; latency
set -o pipefail
mkdir -p gpurun_out/r5s2
T="timeout -k 10"
for i in 1 2; do
  SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/base2/libsrs_amd.so $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5s2/base$i.json 2> gpurun_out/r5s2/base$i.err || exit 1
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5s2/new$i.json 2> gpurun_out/r5s2/new$i.err || exit 2
done
$T 200 python -u tools/latency.py 4096 8193 65536 262144 524288 1048576 4194304 > gpurun_out/r5s2/lat.txt 2>&1 || exit 3
SRS_AMD_LIB=simd-radix-sort_amd/lib/variants/base2/libsrs_amd.so $T 200 python -u tools/latency.py 524288 1048576 4194304 > gpurun_out/r5s2/lat_base.txt 2>&1 || exit 4

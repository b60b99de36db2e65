cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag
for c in c1 c2 c3; do SRS_TRACE_LEVELS=1 timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 1 --cpu-sample 0 --no-verify > gpurun_out/diag/trace_$c.log 2>&1 || exit 1; done
SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/stamps/libsrs_amd.so timeout -k 10 300 python tools/stamps.py > gpurun_out/diag/stamps_c1.log 2>&1

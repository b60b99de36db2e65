cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sweep
i=0
for v in $VARS; do i=$((i+1)); log=gpurun_out/sweep/${CFG:-c1}_${i}_$v.log
SRS_AMD_LIB=$PWD/simd-radix-sort_amd/lib/variants/$v/libsrs_amd.so timeout -k 10 300 python bench.py --n ${N:-1e9} --config ${CFG:-c1} --steps ${STEPS:-5} --cpu-sample 0 $EXTRA > $log 2>&1; rc=$?
echo "$v rc=$rc $(python tools/show.py $log | cut -d' ' -f2-)" | cut -c1-330
[ $rc -ge 124 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc; done; exit 0

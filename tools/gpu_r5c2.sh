# round 5, GPU call c: the default bench line (driver's command), then the
# round profile (kernel trace + HBM counter passes) of the headline
set -o pipefail
mkdir -p gpurun_out/r5c2
T="timeout -k 10"
: # (GPU suite: 306 passed in the r5c call)
t0=$(date +%s)
$T 600 python -u bench.py > gpurun_out/r5c2/bench_default.json 2> gpurun_out/r5c2/bench_default.err || exit 1
echo "bench wall s: $(( $(date +%s) - t0 ))" > gpurun_out/r5c2/bench_wall.txt
bash tools/profile_round.sh r05 --cpu-sample 0 --alloc-steps 0 --steps 10 > gpurun_out/r5c2/prof.log 2>&1 || exit 2

# round 5, GPU call c: the default bench line (driver's command), then the
# round profile (kernel trace + HBM counter passes) of the headline
set -o pipefail
mkdir -p gpurun_out/r5c
T="timeout -k 10"
$T 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5c/t.txt 2>&1 || exit 3
t0=$(date +%s)
$T 600 python -u bench.py > gpurun_out/r5c/bench_default.json 2> gpurun_out/r5c/bench_default.err || exit 1
echo "bench wall s: $(( $(date +%s) - t0 ))" > gpurun_out/r5c/bench_wall.txt
bash tools/profile_round.sh r05 --cpu-sample 0 --alloc-steps 0 --steps 10 > gpurun_out/r5c/prof.log 2>&1 || exit 2

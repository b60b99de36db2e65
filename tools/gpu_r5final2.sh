# round 5, final GPU call B: round profiles of C1 / C2 / C3 (kernel trace +
# FETCH_SIZE + WRITE_SIZE) and the reference-format curves
set -o pipefail
mkdir -p gpurun_out/r5f
T="timeout -k 10"
bash tools/profile_round.sh r05f --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5f/p1.log 2>&1 || exit 3
bash tools/profile_round.sh r05fc2 --config c2 --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5f/p2.log 2>&1 || exit 4
bash tools/profile_round.sh r05fc3 --config c3 --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5f/p3.log 2>&1 || exit 5
$T 600 python -u tools/perf_dat.py --out gpurun_out/r5f/dat --types int64 --payload int64 --dists Uniform --max-log2 22 > gpurun_out/r5f/dat.log 2>&1 || exit 6

# round 5, GPU call j: round profiles (kernel trace + FETCH_SIZE + WRITE_SIZE) of C1, C2, C3
set -o pipefail
mkdir -p gpurun_out/r5j
bash tools/profile_round.sh r05 --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5j/p1.log 2>&1 || exit 1
bash tools/profile_round.sh r05c2 --config c2 --cpu-sample 0 --alloc-steps 0 --steps 10 > gpurun_out/r5j/p2.log 2>&1 || exit 2
bash tools/profile_round.sh r05c3 --config c3 --cpu-sample 0 --alloc-steps 0 --steps 10 > gpurun_out/r5j/p3.log 2>&1 || exit 3

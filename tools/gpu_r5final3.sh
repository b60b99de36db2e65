# round 5, final GPU call B (on the final library): round profiles of C1 / C2 / C3 (kernel trace +
# FETCH_SIZE + WRITE_SIZE) and the reference-format curves
set -o pipefail
mkdir -p gpurun_out/r5g2
T="timeout -k 10"
bash tools/profile_round.sh r05g --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5g2/p1.log 2>&1 || exit 3
bash tools/profile_round.sh r05gc2 --config c2 --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5g2/p2.log 2>&1 || exit 4
bash tools/profile_round.sh r05gc3 --config c3 --cpu-sample 0 --alloc-steps 0 --steps 10 --extra none > gpurun_out/r5g2/p3.log 2>&1 || exit 5

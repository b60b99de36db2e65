# round 5, GPU call k: C2 pair A/B after the staged-digit change; pair tests
set -o pipefail
mkdir -p gpurun_out/r5k
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 300 --timeout-method thread -m gpu -k "tile_pair or two_u32 or float_keys_two" > gpurun_out/r5k/t.txt 2>&1 || exit 1
$T 200 python -u tools/ab_inproc.py --config c2 --env SRS_PAIR_TILES --values 0,2,3 --rounds 9 > gpurun_out/r5k/ab_c2.json 2> gpurun_out/r5k/ab_c2.err || exit 2

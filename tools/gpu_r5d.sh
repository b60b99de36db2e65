# round 5, GPU call d: in-process A/B of the tile-pair scatter (C1, C2, C3),
# the forced-mode pair tests
set -o pipefail
mkdir -p gpurun_out/r5d
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_sort.py -x -v --timeout 300 --timeout-method thread -m gpu -k "tile_pair or two_u32" > gpurun_out/r5d/t.txt 2>&1 || exit 1
$T 200 python -u tools/ab_inproc.py --config c1 --env SRS_PAIR_TILES --values 0,1 --rounds 9 > gpurun_out/r5d/ab_c1.json 2> gpurun_out/r5d/ab_c1.err || exit 2
$T 200 python -u tools/ab_inproc.py --config c2 --env SRS_PAIR_TILES --values 0,2,3 --rounds 9 > gpurun_out/r5d/ab_c2.json 2> gpurun_out/r5d/ab_c2.err || exit 3
$T 200 python -u tools/ab_inproc.py --config c3 --env SRS_PAIR_TILES --values 0,1 --rounds 9 > gpurun_out/r5d/ab_c3.json 2> gpurun_out/r5d/ab_c3.err || exit 4

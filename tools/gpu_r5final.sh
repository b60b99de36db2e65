# round 5, final GPU call A (last rerun of the round): the whole GPU suite, then the default bench line
# (CPU baselines included)
set -o pipefail
mkdir -p gpurun_out/r5j2
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j2/pytest_gpu.txt 2>&1 || exit 1
$T 600 python -u bench.py > gpurun_out/r5j2/bench_default.json 2> gpurun_out/r5j2/bench_default.err || exit 2

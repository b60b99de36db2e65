# round 5, GPU call e: placed vs plain vs in-place outputs after the probe fix
set -o pipefail
mkdir -p gpurun_out/r5e
T="timeout -k 10"
for i in 1 2 3; do
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5e/b$i.json 2> gpurun_out/r5e/b$i.err || exit $i
done

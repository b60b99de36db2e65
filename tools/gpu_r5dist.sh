# round 5: the reference's input distributions at 1e9 (C1 shape) on the final library
set -o pipefail
mkdir -p gpurun_out/r5dist
T="timeout -k 10"
for d in zero zeroone gaussian sorted reverse almostsorted almostreverse; do
  $T 240 python -u bench.py --dist $d --cpu-sample 0 --extra none --alloc-steps 0 --steps 5 > gpurun_out/r5dist/$d.json 2> gpurun_out/r5dist/$d.err || exit 1
done

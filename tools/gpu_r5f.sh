# round 5, GPU call f: placement off (SRS_PLACE=0) vs on, alternating processes
set -o pipefail
mkdir -p gpurun_out/r5f
T="timeout -k 10"
for i in 1 2 3; do
  SRS_PLACE=0 $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 --extra none > gpurun_out/r5f/off$i.json 2> gpurun_out/r5f/off$i.err || exit $i
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 --extra none > gpurun_out/r5f/on$i.json 2> gpurun_out/r5f/on$i.err || exit $i
done

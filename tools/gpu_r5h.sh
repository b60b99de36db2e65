# round 5, GPU call h: placement with the tighter threshold: output A/B and bench lines
set -o pipefail
mkdir -p gpurun_out/r5h
T="timeout -k 10"
$T 300 python -u tools/ab_outputs.py --sets placed,plain,placed,plain,placed,plain > gpurun_out/r5h/ab1.json 2> gpurun_out/r5h/ab1.err || exit 1
for i in 1 2 3; do
  $T 300 python -u bench.py --cpu-sample 0 --cpu-sample-extra 0 > gpurun_out/r5h/b$i.json 2> gpurun_out/r5h/b$i.err || exit 2
done

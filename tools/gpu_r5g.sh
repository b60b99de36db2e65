# round 5, GPU call g: output-buffer A/B in one process (placed vs plain), two processes
set -o pipefail
mkdir -p gpurun_out/r5g
T="timeout -k 10"
for i in 1 2; do
  $T 300 python -u tools/ab_outputs.py --sets placed,plain,placed,plain,plain,placed > gpurun_out/r5g/ab$i.json 2> gpurun_out/r5g/ab$i.err || exit $i
done

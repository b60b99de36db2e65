# round 5, GPU call b: the whole GPU suite, C2 tile-pair A/B, shard world-1 lines
set -o pipefail
mkdir -p gpurun_out/r5b2
T="timeout -k 10"
: # (tests passed in the first r5b call)
for i in 1 2; do
  SRS_PAIR_TILES=0 $T 200 python -u bench.py --config c2 --steps 10 --cpu-sample 0 --extra none --alloc-steps 0 > gpurun_out/r5b2/c2_off_$i.json 2>gpurun_out/r5b2/c2_off_$i.err || exit 2
  $T 200 python -u bench.py --config c2 --steps 10 --cpu-sample 0 --extra none --alloc-steps 0 > gpurun_out/r5b2/c2_on_$i.json 2>gpurun_out/r5b2/c2_on_$i.err || exit 3
done
for i in 1 2; do
  $T 200 python -u bench.py --config c1 --steps 10 --cpu-sample 0 --extra none --alloc-steps 0 > gpurun_out/r5b2/c1_def_$i.json 2>gpurun_out/r5b2/c1_def_$i.err || exit 6
  SRS_PAIR_TILES=1 $T 200 python -u bench.py --config c1 --steps 10 --cpu-sample 0 --extra none --alloc-steps 0 > gpurun_out/r5b2/c1_pair_$i.json 2>gpurun_out/r5b2/c1_pair_$i.err || exit 7
done
$T 300 python -u bench.py --shard --steps 5 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0 > gpurun_out/r5b2/shard_w1_default.json 2> gpurun_out/r5b2/shard_w1_default.err || exit 4
$T 300 python -u bench.py --shard --steps 5 --warmup 1 --cpu-sample 0 --extra none --alloc-steps 0 --rounds 16 --chunks 8 > gpurun_out/r5b2/shard_w1_r16c8.json 2> gpurun_out/r5b2/shard_w1_r16c8.err || exit 5

#!/bin/bash
# Round-3 final tree: every -m gpu test, smoke, the driver's bench command, the 10B / 200B / 100M
# pipelined lines, a kernel trace of the bench, PMC passes of the north-star step, the P = 8 sim
export TMPDIR=/tmp
TAG=${1:-r03f}
bash tools/gpu_round.sh $TAG tests smoke bench prof || exit 1
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for C in 10b 200b 100m; do
  timeout -k 10 180 python bench.py --config $C $B > gpurun_out/bench_${C}_${TAG}.json 2> gpurun_out/bench_${C}_${TAG}.err || exit 1
done
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 10 > gpurun_out/sim_P8_${TAG}.json 2> gpurun_out/sim_P8_${TAG}.err || exit 1
bash tools/pmc_passes.sh nstar ${TAG}_nstar rd wr dram valu stall

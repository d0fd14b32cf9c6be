#!/bin/bash
# Include? route from SHA-1 words hashed by the previous step's owner test (--dig): parity, then
# P = 8 north-star and 200B x 8 per-rank steps with and without it, interleaved
export TMPDIR=/tmp
TAG=${1:-r03aa}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py -k "chunked" > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for D in "" "--dig"; do
    timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 $D > gpurun_out/sim_P8${D/--/_}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
    timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b $D > gpurun_out/sim_200b${D/--/_}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done

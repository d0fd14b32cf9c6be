#!/bin/bash
# Side hash in the L2 sweep with LDS-staged keys: parity, then P = 8 --dig vs none
export TMPDIR=/tmp
TAG=${1:-r03ad}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py -k "chunked" > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for D in "" "--dig"; do
    N=$(echo "$D" | tr -d ' -'); N=${N:-none}
    timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 10 $D > gpurun_out/sim_P8_${N}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done

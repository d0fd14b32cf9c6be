#!/bin/bash
# L2 sweep grid (resident workgroups: 1024 = 4 per CU, 2048 = 8 per CU) with the XCD-local order
export TMPDIR=/tmp
TAG=${1:-r03ae}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py -k "chunked and l2" > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for G in ${GRIDS:-1024 1536 2048}; do
    BFHIP_L2_GRID=$G timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 10 > gpurun_out/sim_P8_g${G}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done

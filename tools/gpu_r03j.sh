#!/bin/bash
# L2-local owner test: grid size A/B at P = 8 (512 route buckets: 4 MiB superbins), sorted test beside
export TMPDIR=/tmp
TAG=${1:-r03j}
for G in 256 512 1024; do
  BFHIP_CHUNK_TEST_L2=1 BFHIP_CHUNK_BUCKETS=512 BFHIP_L2_GRID=$G timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
      > gpurun_out/sim_l2g${G}_P8_${TAG}.json 2> gpurun_out/sim_l2g${G}_P8_${TAG}.err || exit 1
done
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_sorted_P8_${TAG}.json 2> gpurun_out/sim_sorted_P8_${TAG}.err || exit 1

#!/bin/bash
# 200B x 8 owner include?: the XCD-local L2 sweep forced (its superbins are larger than 4 MiB
# there) against the keyed mid + bin_test the auto choice takes
export TMPDIR=/tmp
TAG=${1:-r03ag}
for i in 1 2; do
  for L in 2 1; do
    BFHIP_CHUNK_TEST_L2=$L timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_200b_l2${L}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done
for B in 256 512; do
  BFHIP_CHUNK_TEST_L2=1 BFHIP_CHUNK_BUCKETS=$B timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_200b_l21_b${B}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
done

#!/bin/bash
# L2-local owner test: grid / bucket A/B at P = 8, and the 200B x8 shard with it
export TMPDIR=/tmp
TAG=${1:-r03k}
BFHIP_L2_GRID=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
    -k "chunked and l2" > gpurun_out/tests_l2_${TAG}.log 2>&1 || { echo "l2 tests failed"; exit 1; }
for V in "768 512" "1024 512" "1280 512" "1536 512" "1024 256"; do
  set -- $V
  BFHIP_CHUNK_TEST_L2=1 BFHIP_CHUNK_BUCKETS=$2 BFHIP_L2_GRID=$1 timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
      > gpurun_out/sim_l2g$1_b$2_P8_${TAG}.json 2> gpurun_out/sim_l2_P8_${TAG}.err || exit 1
done
for V in "0 256 1024" "1 512 1024"; do
  set -- $V
  BFHIP_CHUNK_TEST_L2=$1 BFHIP_CHUNK_BUCKETS=$2 BFHIP_L2_GRID=$3 timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b \
      > gpurun_out/sim_200b_l2$1_b$2_${TAG}.json 2> gpurun_out/sim_200b_${TAG}.err || exit 1
done
REPS=8 timeout -k 10 180 python tools/host_api_bench.py > gpurun_out/host_api_${TAG}.json 2> gpurun_out/host_api_${TAG}.err || exit 1

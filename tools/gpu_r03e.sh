#!/bin/bash
# chunk tests (direct / sorted / L2 owners), P = 8 sims: L2 test vs sorted test, 512 vs 256 buckets
export TMPDIR=/tmp
TAG=${1:-r03e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
    -k "chunked" > gpurun_out/tests_chunks_${TAG}.log 2>&1 || { echo "chunk tests failed"; exit 1; }
for V in "L2=1 B=512" "L2=0 B=256" "L2=1 B=256"; do
  set -- $V; L=${1#L2=}; B=${2#B=}
  BFHIP_CHUNK_TEST_L2=$L BFHIP_CHUNK_BUCKETS=$B timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
      > gpurun_out/sim_l2${L}_b${B}_P8_${TAG}.json 2> gpurun_out/sim_l2${L}_b${B}_P8_${TAG}.err || exit 1
done
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_ch_P8_200b_${TAG}.json 2> gpurun_out/sim_ch_P8_200b_${TAG}.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_merged.py -x -v --timeout 280 --timeout-method thread > gpurun_out/tests_merged_${TAG}.log 2>&1 || { echo "merged test failed"; exit 1; }
for G in keys digests; do
  timeout -k 10 180 python tools/sim_rank.py --replicated 8 --gathered $G --config 10b --steps 3 > gpurun_out/sim_repl8_${G}_${TAG}.json 2> gpurun_out/sim_repl8_${G}_${TAG}.err || exit 1
done

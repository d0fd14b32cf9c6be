#!/bin/bash
# r03 GPU pass: the chunked-window primitives and every multi-rank test, then the P = 8
# per-rank sims (chunked vs plain sync-free windows).  gpurun -- bash tools/gpu_r03.sh <tag>
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
    -k "chunked" > gpurun_out/tests_chunks_${TAG}.log 2>&1 || { echo "chunk tests failed"; exit 1; }
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_ch_P8_${TAG}.json 2> gpurun_out/sim_ch_P8_${TAG}.err || exit 1
timeout -k 10 120 python tools/sim_rank.py --shards 8 --sync-free --steps 5 > gpurun_out/sim_sf_P8_${TAG}.json 2> gpurun_out/sim_sf_P8_${TAG}.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_distributed.py tests/test_gpu_dist_gloo.py \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_dist_${TAG}.log 2>&1 || { echo "dist tests failed"; exit 1; }

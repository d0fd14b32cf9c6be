#!/bin/bash
# auto chunk geometry (L2 sweep at <= 4 MiB superbins): parity, P = 8 / 200B sims, then r03l's A/Bs
export TMPDIR=/tmp
TAG=${1:-r03m}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py tests/test_gpu_dist_gloo.py > gpurun_out/tests_chunks_${TAG}.log 2>&1 || exit 1
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_auto_P8_${TAG}.json 2> gpurun_out/sim_auto_P8_${TAG}.err || exit 1
timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_auto_200b_${TAG}.json 2> gpurun_out/sim_auto_200b_${TAG}.err || exit 1
bash tools/gpu_r03l.sh $TAG

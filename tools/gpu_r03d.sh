#!/bin/bash
# chunk tests, P = 8 sims (route buckets 512 vs 256), XCD-local probe rates, host-API prefault A/B
export TMPDIR=/tmp
TAG=${1:-r03d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
    -k "chunked" > gpurun_out/tests_chunks_${TAG}.log 2>&1 || { echo "chunk tests failed"; exit 1; }
for B in 512 256; do
  BFHIP_CHUNK_BUCKETS=$B timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_ch${B}_P8_${TAG}.json 2> gpurun_out/sim_ch${B}_P8_${TAG}.err || exit 1
done
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_ch_P8_200b_${TAG}.json 2> gpurun_out/sim_ch_P8_200b_${TAG}.err || exit 1
timeout -k 10 60 ./tools/probe_xcd > gpurun_out/probe_xcd_${TAG}.log 2>&1 || exit 1
REPS=8 timeout -k 10 180 python tools/host_api_bench.py > gpurun_out/host_api_${TAG}.json 2> gpurun_out/host_api_${TAG}.err || exit 1

#!/bin/bash
# Host-pointer path: host staging threads 8 / 16 / 32 (BFHIP_HOST_THREADS), and chunk size
export TMPDIR=/tmp
TAG=${1:-r03h2}
for T in 16 8 32; do
  BFHIP_HOST_THREADS=$T REPS=6 timeout -k 10 180 python tools/host_api_bench.py > gpurun_out/host_t${T}_${TAG}.json 2> gpurun_out/host_${TAG}.err || exit 1
done

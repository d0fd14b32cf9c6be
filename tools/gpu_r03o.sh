#!/bin/bash
# Persistent pipelined bin_apply (bin_apply_pipe_kernel): binned parity, then interleaved A/B
# against bin_apply_kernel (BFHIP_APPLY_PIPE_GRID=0) on the 10B and north-star steps
export TMPDIR=/tmp
TAG=${1:-r03o}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py tests/test_gpu_digests.py -k "binned or merged or digest or 200b or pipelined" \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for G in 0 ""; do
    for C in 10b nstar; do
      BFHIP_APPLY_PIPE_GRID=$G timeout -k 10 120 python bench.py --config $C $B > gpurun_out/ab_${C}_g${G:-def}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
    done
  done
done

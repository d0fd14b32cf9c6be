#!/bin/bash
# Two-workgroup-per-CU wide digest front (k > 12: 10B / 200B) against one per CU (BFHIP_FRONT_WIDE2=0)
export TMPDIR=/tmp
TAG=${1:-r03ac}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_digests.py tests/test_gpu_parity.py -k "digest or 200b or k13 or k16 or pipelined" \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for W in 0 1; do
    BFHIP_FRONT_WIDE2=$W timeout -k 10 120 python bench.py --config 10b $B > gpurun_out/ab_10b_w${W}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
  done
done

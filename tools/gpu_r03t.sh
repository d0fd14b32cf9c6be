#!/bin/bash
# 64-B sector stores in the line-dense apply (BFHIP_APPLY_FRESH=2) against fresh 16-B vectors (1)
export TMPDIR=/tmp
TAG=${1:-r03t}
BFHIP_APPLY_FRESH=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py -k "binned or merged or 200b" \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for F in 1 2; do
    BFHIP_APPLY_FRESH=$F timeout -k 10 120 python bench.py --config 10b $B > gpurun_out/ab_10b_fr${F}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
  done
done
export BFHIP_APPLY_FRESH=2
bash tools/pmc_passes.sh 10b r03t_10b wr
timeout -k 10 180 python tools/cu_mask_probe.py > gpurun_out/cu_mask_${TAG}.jsonl 2> gpurun_out/cu_mask_${TAG}.err || exit 1

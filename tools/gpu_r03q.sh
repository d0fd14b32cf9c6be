#!/bin/bash
# Dense apply forms A/B (BFHIP_APPLY_FORM 0 bin_apply, 1 pipe, 2 tab-prefetch) + binned parity under form 2
export TMPDIR=/tmp
TAG=${1:-r03q}
BFHIP_APPLY_FORM=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py -k "binned or merged or 200b" \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for F in 0 1 2; do
    for C in 10b nstar; do
      BFHIP_APPLY_FORM=$F timeout -k 10 120 python bench.py --config $C $B > gpurun_out/ab_${C}_f${F}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
    done
  done
done

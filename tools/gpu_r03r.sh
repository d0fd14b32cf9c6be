#!/bin/bash
# Host-path D2H stream (ab_libs/d2h_old = before) A/B, dense apply forms A/B, their parity tests
export TMPDIR=/tmp
TAG=${1:-r03r}
BFHIP_APPLY_FORM=2 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py tests/test_gpu_per_key.py tests/test_gpu_multi.py \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for L in old new; do
    if [ $L = old ]; then LIB=$PWD/ab_libs/d2h_old/libbfhip.so; else LIB=$PWD/redis-bloomfilter_amd/lib/libbfhip.so; fi
    BFHIP_LIB=$LIB REPS=6 timeout -k 10 180 python tools/host_api_bench.py > gpurun_out/host_${L}_${i}_${TAG}.json 2> gpurun_out/host_${TAG}.err || exit 1
  done
done
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for F in 0 1 2; do
    for C in 10b nstar; do
      BFHIP_APPLY_FORM=$F timeout -k 10 120 python bench.py --config $C $B > gpurun_out/ab_${C}_f${F}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
    done
  done
done

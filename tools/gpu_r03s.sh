#!/bin/bash
# XCD-aware region order in bin_apply / bin_test / the pipelined apply: parity, then A/B
# against the tree before it (ab_libs/noxcd), 10B and north-star steps, interleaved
export TMPDIR=/tmp
TAG=${1:-r03s}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py tests/test_gpu_digests.py tests/test_gpu_distributed.py \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for L in noxcd xcd; do
    if [ $L = noxcd ]; then LIB=$PWD/ab_libs/noxcd/libbfhip.so; else LIB=$PWD/redis-bloomfilter_amd/lib/libbfhip.so; fi
    for C in 10b nstar; do
      BFHIP_LIB=$LIB timeout -k 10 120 python bench.py --config $C $B > gpurun_out/ab_${C}_${L}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
    done
  done
done

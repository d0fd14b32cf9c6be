#!/bin/bash
# XCD-grouped bin_mid / bin_mid_chunks (ab_libs/midold: superbins spread over the XCDs)
export TMPDIR=/tmp
TAG=${1:-r03y}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_merged.py tests/test_gpu_distributed.py -k "binned or merged or 200b or chunk or shard" \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
B="--steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
for i in 1 2; do
  for L in midold new; do
    if [ $L = midold ]; then LIB=$PWD/ab_libs/midold/libbfhip.so; else LIB=$PWD/redis-bloomfilter_amd/lib/libbfhip.so; fi
    for C in 10b nstar; do
      BFHIP_LIB=$LIB timeout -k 10 120 python bench.py --config $C $B > gpurun_out/ab_${C}_${L}_${i}_${TAG}.json 2> gpurun_out/ab_${TAG}.err || exit 1
    done
    BFHIP_LIB=$LIB timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_P8_${L}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done
export BFHIP_LIB=$PWD/redis-bloomfilter_amd/lib/libbfhip.so
bash tools/pmc_passes.sh 10b ${TAG}_10b wr

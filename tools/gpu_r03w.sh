#!/bin/bash
# XCD-local L2 sweep of the chunked owner include? (ab_libs/l2old: whole-grid sweep): parity,
# then P = 8 north-star and 200B x 8 per-rank steps, interleaved
export TMPDIR=/tmp
TAG=${1:-r03w}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_distributed.py tests/test_gpu_dist_gloo.py > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for L in l2old new; do
    if [ $L = l2old ]; then LIB=$PWD/ab_libs/l2old/libbfhip.so; else LIB=$PWD/redis-bloomfilter_amd/lib/libbfhip.so; fi
    BFHIP_LIB=$LIB timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_P8_${L}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
    BFHIP_LIB=$LIB timeout -k 10 180 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b > gpurun_out/sim_200b_${L}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --output-format csv -d gpurun_out/pmc_${TAG}_P8_rw -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_rw.log 2>&1 || exit 1

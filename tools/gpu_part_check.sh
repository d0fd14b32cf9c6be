#!/bin/bash
# Binned-kernel change check: parity + distributed tests, the per-rank compute simulation at
# P = 8 and 4 (tools/sim_sf.sh), and a short north-star bench.
#   gpurun -- bash tools/gpu_part_check.sh <tag>
export TMPDIR=/tmp
TAG=${1:-part}
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_distributed.py tests/test_gpu_dist_gloo.py}
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -k "not rehearsal" \
    > gpurun_out/tests_${TAG}.log 2>&1 &&
bash tools/sim_sf.sh &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api \
    --no-reference-shapes > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err

#!/bin/bash
# after the any_new fix: nstar bench (driver form), 10B bench with 512 / 256 superbins, the
# replicated x8 proxy, and the multi-device / digest tests
export TMPDIR=/tmp
TAG=${1:-r03h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/tests_flags_${TAG}.log 2>&1 || { echo "flag tests failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-reference-shapes \
    > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit 1
for S in 512 256; do
  BFHIP_BIN_MAX_SUP=$S timeout -k 10 240 python bench.py --config 10b --steps 10 --warmup 3 --no-secondary --no-cpu-baseline \
      --no-host-api --no-reference-shapes > gpurun_out/bench10b_sup${S}_${TAG}.json 2> gpurun_out/bench10b_sup${S}_${TAG}.err || exit 1
done
for G in digests keys; do
  timeout -k 10 240 python tools/sim_rank.py --replicated 8 --gathered $G --config 10b --steps 3 > gpurun_out/sim_repl8_${G}_${TAG}.json 2> gpurun_out/sim_repl8_${TAG}.err || exit 1
done

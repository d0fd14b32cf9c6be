#!/bin/bash
# parity of the 512-superbin / hierarchical-scan plans, then A/B: balanced superbins at 10B
# (bench --config 10b), the replicated x8 proxy, and the side-stream route overlap at P = 8
export TMPDIR=/tmp
TAG=${1:-r03g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_merged.py -x -v --timeout 280 --timeout-method thread \
    -k "binned_edge or 200b or 10b or merged or config" > gpurun_out/tests_plans_${TAG}.log 2>&1 || { echo "plan tests failed"; exit 1; }
for S in 512 256; do
  BFHIP_BIN_MAX_SUP=$S timeout -k 10 240 python bench.py --config 10b --steps 10 --warmup 3 --no-secondary --no-cpu-baseline \
      --no-host-api --no-reference-shapes > gpurun_out/bench10b_sup${S}_${TAG}.json 2> gpurun_out/bench10b_sup${S}_${TAG}.err || exit 1
done
timeout -k 10 240 python tools/sim_rank.py --replicated 8 --gathered digests --config 10b --steps 3 > gpurun_out/sim_repl8_digests_${TAG}.json 2> gpurun_out/sim_repl8_${TAG}.err || exit 1
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_ch_P8_${TAG}.json 2> gpurun_out/sim_ch_P8_${TAG}.err || exit 1
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --overlap --steps 5 > gpurun_out/sim_chov_P8_${TAG}.json 2> gpurun_out/sim_chov_P8_${TAG}.err || exit 1

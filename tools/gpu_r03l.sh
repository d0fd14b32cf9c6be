#!/bin/bash
# 10B apply: store only fresh vectors (A/B, interleaved); the replicated step's host wait at world 1
# over RCCL (sizes pipelined one batch ahead)
export TMPDIR=/tmp
TAG=${1:-r03l}
for R in 1 2; do for F in 0 1; do
  BFHIP_APPLY_FRESH=$F timeout -k 10 240 python bench.py --config 10b --steps 10 --warmup 3 --no-secondary --no-cpu-baseline \
      --no-host-api --no-reference-shapes > gpurun_out/bench10b_fresh${F}_${R}_${TAG}.json 2> gpurun_out/bench10b_${TAG}.err || exit 1
done; done
timeout -k 10 240 python bench.py --mode replicated --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --no-host-api \
    --no-reference-shapes > gpurun_out/bench_repl1_${TAG}.json 2> gpurun_out/bench_repl1_${TAG}.err || exit 1

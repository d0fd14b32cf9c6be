#!/bin/bash
# Replicated layout (world 1 over RCCL, the N >= 2 code path): kernel trace of the timed steps,
# to read the GPU's idle gaps between steps
export TMPDIR=/tmp
TAG=${1:-r03i2}
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}_repl -o run -- \
    python bench.py --mode replicated --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --no-host-api \
    --no-reference-shapes > gpurun_out/bench_repl_${TAG}.json 2> gpurun_out/bench_repl_${TAG}.err || exit 1

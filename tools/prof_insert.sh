#!/bin/bash
# Kernel-trace profile of the north-star bench (binned insert on, the default)
# plus an A/B run with the direct insert; run on the GPU box from the repo root.
export TMPDIR=/tmp
BENCH="python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_binned -o run -- \
    $BENCH > gpurun_out/b_binned.json 2> gpurun_out/b_binned.err &&
BFHIP_INSERT_BINNED=0 timeout -k 10 120 $BENCH > gpurun_out/b_direct.json 2> gpurun_out/b_direct.err

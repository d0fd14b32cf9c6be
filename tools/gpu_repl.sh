#!/bin/bash
# Replicated layout on the GPU box: world-1 RCCL tests and the replicated bench at world size 1.
export TMPDIR=/tmp
T=${1:-r}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread -k "world1" \
    > gpurun_out/${T}_tests.log 2>&1 &&
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533" &&
B="bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes" &&
timeout -k 10 200 $R $B --mode replicated > gpurun_out/${T}_repl_N1.json 2> gpurun_out/${T}_repl_N1.err

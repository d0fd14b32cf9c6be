#!/bin/bash
# Distributed GPU tests + per-rank simulations (window route) + partitioned bench at N=1.
export TMPDIR=/tmp
T=${1:-d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 120 python tools/sim_rank.py --shards 8 --windows > gpurun_out/${T}_sim_P8.json 2> gpurun_out/${T}_sim_P8.err &&
timeout -k 10 120 python tools/sim_rank.py --shards 2 --windows > gpurun_out/${T}_sim_P2.json 2> gpurun_out/${T}_sim_P2.err &&
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533" &&
B="bench.py --mode partitioned --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes" &&
timeout -k 10 200 $R $B > gpurun_out/${T}_part_N1.json 2> gpurun_out/${T}_part_N1.err

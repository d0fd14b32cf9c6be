#!/bin/bash
# BASELINE's multi-GPU layouts through bench.py, rehearsed over gloo with every rank on the
# box's one GPU (correctness of the N > 1 step end to end; the times are not performance
# numbers): configs[3] 10B replicated at N = 2, configs[4] 200B partitioned at N = 4.
export TMPDIR=/tmp
A="--steps 2 --warmup 1 --dist-backend gloo --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --config 10b $A > gpurun_out/rehearse_10b_N2.json 2> gpurun_out/rehearse_10b_N2.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 4 --config 200b $A > gpurun_out/rehearse_200b_N4.json 2> gpurun_out/rehearse_200b_N4.err

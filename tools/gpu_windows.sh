#!/bin/bash
# Window route on the GPU box: partitioned tests, per-rank simulation at P=8 and P=2 with
# and without windows, and the partitioned bench at world size 1 (both routes).
export TMPDIR=/tmp
T=${1:-win}
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 &&
for P in 8 2; do
    timeout -k 10 120 python tools/sim_rank.py --shards $P > gpurun_out/${T}_sim_P${P}_contig.json 2> gpurun_out/${T}_sim_P${P}_contig.err &&
    timeout -k 10 120 python tools/sim_rank.py --shards $P --windows > gpurun_out/${T}_sim_P${P}_win.json 2> gpurun_out/${T}_sim_P${P}_win.err || exit 1
done &&
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533" &&
B="bench.py --mode partitioned --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes" &&
timeout -k 10 200 $R $B > gpurun_out/${T}_part_N1.json 2> gpurun_out/${T}_part_N1.err

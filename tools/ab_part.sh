#!/bin/bash
# A/B of library builds on the partitioned path (world size 1 under torch.distributed.run):
#   bash tools/ab_part.sh <config> <tag>   -> gpurun_out/abp_<tag>_{base,<variant>}.json
export TMPDIR=/tmp
CFG=${1:-nstar}; TAG=${2:-p}
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
B="bench.py --mode partitioned --config $CFG --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
timeout -k 10 200 $R $B > gpurun_out/abp_${TAG}_base.json 2> gpurun_out/abp_${TAG}_base.err || exit 1
for v in redis-bloomfilter_amd/lib/variants/*.so; do
    BFHIP_LIB=$PWD/$v timeout -k 10 200 $R $B > gpurun_out/abp_${TAG}_$(basename $v .so).json \
        2> gpurun_out/abp_${TAG}_$(basename $v .so).err || exit 1
done

#!/bin/bash
# sim_rank.py under env variants:  bash tools/sim_ab.sh <tag> <shards> "ENV=v ..." ...
export TMPDIR=/tmp
TAG=$1; P=$2; shift 2
i=0
for v in "$@"; do
    echo "variant $i: $v" >> gpurun_out/sim_${TAG}.txt
    env $v timeout -k 10 120 python tools/sim_rank.py --shards $P $SIMARGS > gpurun_out/sim_${TAG}_$i.json 2> gpurun_out/sim_${TAG}_$i.err || exit 1
    i=$((i + 1))
done

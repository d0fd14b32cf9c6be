#!/bin/bash
# include? probe-round policy A/B through the native bench (env knobs, no rebuild):
#   bash tools/ab_rounds.sh <config> <tag> "FIRST NEXT" ...
CFG=$1; TAG=$2; shift 2
for v in "$@"; do
    set -- $v
    BFHIP_INCLUDE_FIRST_ROUND=$1 BFHIP_INCLUDE_NEXT_ROUND=$2 timeout -k 10 120 \
        ./redis-bloomfilter_amd/lib/bfbench --config $CFG --steps 10 --warmup 3 \
        > gpurun_out/rounds_${TAG}_${CFG}_$1_$2.json 2> gpurun_out/rounds_${TAG}_${CFG}_$1_$2.err || exit 1
done

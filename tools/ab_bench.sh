#!/bin/bash
# A/B bench variants on the GPU box (from the repo root):
#   bash tools/ab_bench.sh <tag> "ENV=val ENV2=val" "ENV=val" ...
# Each variant runs the north-star bench once (no secondary / CPU / host-API legs)
# and writes gpurun_out/ab_<tag>_<i>.json; a kernel-trace profile of variant 0
# goes to gpurun_out/prof_ab_<tag>.
export TMPDIR=/tmp
TAG=$1; shift
BENCH="python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes ${BENCH_EXTRA:-}"
i=0
for v in "$@"; do
    echo "variant $i: $v" >> gpurun_out/ab_${TAG}.txt
    env $v timeout -k 10 120 $BENCH > gpurun_out/ab_${TAG}_${i}.json 2> gpurun_out/ab_${TAG}_${i}.err || exit 1
    i=$((i + 1))
done

#!/bin/bash
# P = 8: next include? batch hashed beside the owner test on a second stream (--dig-side) vs
# inside it (--dig) vs the route hashing (none); wall time per step
export TMPDIR=/tmp
TAG=${1:-r03ab}
for i in 1 2; do
  for D in "" "--dig" "--dig --dig-side"; do
    N=$(echo "$D" | tr -d ' -'); N=${N:-none}
    timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 10 $D > gpurun_out/sim_P8_${N}_${i}_${TAG}.json 2> gpurun_out/sim_${TAG}.err || exit 1
  done
done

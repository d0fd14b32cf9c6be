#!/bin/bash
# Round 4: the P = 8 per-rank step (time, stall/LDS and VALU counters of its kernels), and
# the owner mid's load depth A/B on it.  A failing step ends the script.
export TMPDIR=/tmp
TAG=${1:-r04c}
bash tools/gpu_round.sh $TAG simP8 || exit $?
for d in 1 2 1 2; do
    BFHIP_MID_DEPTH=$d timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
        > gpurun_out/sim_P8_mid${d}_${TAG}.json 2>/dev/null || exit $?
    (echo -n "{\"depth\": $d, \"line\": "; cat gpurun_out/sim_P8_mid${d}_${TAG}.json; echo "}") >> gpurun_out/sim_P8_mid_${TAG}.jsonl
done

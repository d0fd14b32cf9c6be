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
# the region-set kernels' counters (10B x 8 replicated sim, sets form)
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
            "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_INSTS_SMEM"; do
    n=$((n + 1))
    timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc_${TAG}_sets_$n -o run -- \
        python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --steps 1 \
        > gpurun_out/pmc_${TAG}_sets_$n.log 2>&1 || exit $?
done

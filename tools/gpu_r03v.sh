#!/bin/bash
# P = 8 chunked per-rank step: time, then VALU and stall counters per kernel
export TMPDIR=/tmp
TAG=${1:-r03v}
timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 > gpurun_out/sim_P8_${TAG}.json 2> gpurun_out/sim_P8_${TAG}.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
    --output-format csv -d gpurun_out/pmc_${TAG}_P8_stall -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_stall.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d gpurun_out/pmc_${TAG}_P8_valu -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_valu.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --output-format csv -d gpurun_out/pmc_${TAG}_P8_rw -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_rw.log 2>&1 || exit 1

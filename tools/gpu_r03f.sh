#!/bin/bash
# counters of the merged (replicated x8) 10B insert: where bin_apply's time goes; plus the
# chunked P = 8 / 200B sims with the sorted owner test (L2 sweep off)
export TMPDIR=/tmp
TAG=${1:-r03f}
run() {   # pass, counters...
    local pass=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_${pass} -o run -- \
        python tools/sim_rank.py --replicated 8 --gathered digests --config 10b --steps 1 \
        > gpurun_out/pmc_${TAG}_${pass}.log 2>&1
}
run stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS || exit 1
run mem TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU || exit 1
for V in "0 256" "0 512"; do
  set -- $V
  BFHIP_CHUNK_TEST_L2=$1 BFHIP_CHUNK_BUCKETS=$2 timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 --config 200b \
      > gpurun_out/sim_ch_P8_200b_l2$1_b$2_${TAG}.json 2> gpurun_out/sim_ch_P8_200b_${TAG}.err || exit 1
done

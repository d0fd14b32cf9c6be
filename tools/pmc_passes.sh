#!/bin/bash
# PMC passes over the bench's north-star workload (run on the GPU box from the
# repo root).  One rocprofv3 run per counter group (gfx950: <= 4 TCC counters
# per pass), kernel trace kept separate; outputs under gpurun_out/pmc_<tag>/.
# Summarise with: python tools/pmc_summary.py gpurun_out/pmc_* > profiles/...
export TMPDIR=/tmp
CMD="python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-host-api"
run() {   # tag, counters...
    local tag=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${tag} -o run -- $CMD \
        > gpurun_out/pmc_${tag}.log 2>&1
}
run rd   TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_64B_sum &&
run wr   TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_128B_sum &&
run dram TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum &&
run fs   FETCH_SIZE &&
run ws   WRITE_SIZE

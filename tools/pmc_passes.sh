#!/bin/bash
# PMC passes over one bench workload (run on the GPU box from the repo root):
#   bash tools/pmc_passes.sh [config] [tag] [passes...]
# One rocprofv3 run per counter group (gfx950: <= 4 TCC, <= 8 SQ, <= 2 GRBM counters per
# pass), kernel trace kept separate; outputs under gpurun_out/pmc_<tag>_<pass>/.
# Summarise with: python tools/pmc_summary.py gpurun_out/pmc_<tag>_* --workload <config>
export TMPDIR=/tmp
CONFIG=${1:-nstar}
TAG=${2:-$CONFIG}
if [ $# -gt 2 ]; then shift 2; PASSES="$*"; else PASSES="rd wr dram valu"; fi
# lua_1m: the Lua layout's secondary alone (bench.py lua_config), behind the tiny 10k config
# model_*: the per-rank models of bench.py's multi_gpu_models legs (tools/sim_rank.py, the same
# argv as bench.MODEL_LEGS with fewer steps)
PROG="bench.py"
case "$CONFIG" in
    lua_1m) BENCH_ARGS="--config 10k --secondary lua_1m --models none --steps 3 --warmup 1 --no-cpu-baseline --no-host-api --no-reference-shapes" ;;
    model_P8_nstar) PROG="tools/sim_rank.py"; BENCH_ARGS="--shards 8 --chunks --config nstar --steps 2" ;;
    model_P8_200b) PROG="tools/sim_rank.py"; BENCH_ARGS="--shards 8 --chunks --config 200b --steps 2" ;;
    model_repl8_10b) PROG="tools/sim_rank.py"; BENCH_ARGS="--replicated 8 --config 10b --gathered sets --fused-hash --overlap-encode apply --steps 2" ;;
    *) BENCH_ARGS="--config $CONFIG --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes" ;;
esac
run() {   # pass, counters...
    local pass=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${TAG}_${pass} -o run -- \
        python $PROG $BENCH_ARGS > gpurun_out/pmc_${TAG}_${pass}.log 2>&1
}
for p in $PASSES; do
    case $p in
        rd)   run rd   TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_64B_sum ;;
        wr)   run wr   TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_128B_sum ;;
        dram) run dram TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum ;;
        valu) run valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT ;;
        stall) run stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
                         SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS ;;
        fs)   run fs   FETCH_SIZE ;;
        ws)   run ws   WRITE_SIZE ;;
    esac || exit $?
done

#!/bin/bash
# Full GPU-box pass: every -m gpu test, smoke(), the driver's bench command, a kernel-trace
# profile of the bench, and the PMC passes (tools/pmc_passes.sh).
# Run from the repo root: gpurun -- bash tools/gpu_round.sh <tag> [steps...]
#   steps: tests smoke bench prof pmc (default: all); also simP8 (the P = 8 per-rank step:
#   time + stall/LDS + VALU counters), repl (one replica's step of the replicated 10B x 8 and
#   north-star x 2 layouts, per insert form)
export TMPDIR=/tmp
TAG=${1:-round}
shift
STEPS=${*:-tests smoke bench prof pmc}
for st in $STEPS; do
    case $st in
        tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
                   ${PYTEST_EXTRA:-} > gpurun_out/tests_${TAG}.log 2>&1 ;;
        smoke) timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_${TAG}.log 2>&1 ;;
        bench) timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
                   > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err ;;
        prof)  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
                   python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes \
                   > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err ;;
        pmc)   bash tools/pmc_passes.sh nstar ${TAG}_nstar ;;
        simP8) timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
                   > gpurun_out/sim_P8_${TAG}.json 2> gpurun_out/sim_P8_${TAG}.err &&
               timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                   SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv \
                   -d gpurun_out/pmc_${TAG}_P8_stall -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 \
                   > gpurun_out/pmc_${TAG}_P8_stall.log 2>&1 &&
               timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES \
                   GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv \
                   -d gpurun_out/pmc_${TAG}_P8_valu -o run -- python tools/sim_rank.py --shards 8 --chunks --steps 2 \
                   > gpurun_out/pmc_${TAG}_P8_valu.log 2>&1 ;;
        repl)  for g in digests sets "sets --fused-hash"; do
                   timeout -k 10 240 python tools/sim_rank.py --replicated 8 --config 10b --gathered $g --steps 3 \
                       >> gpurun_out/sim_repl_${TAG}.jsonl 2>> gpurun_out/sim_repl_${TAG}.err || exit 1
               done &&
               for g in keys sets "sets --fused-hash"; do
                   timeout -k 10 120 python tools/sim_rank.py --replicated 2 --config nstar --gathered $g --steps 5 \
                       >> gpurun_out/sim_repl_${TAG}.jsonl 2>> gpurun_out/sim_repl_${TAG}.err || exit 1
               done ;;
    esac || { echo "step $st failed: $?"; exit 1; }
done

#!/bin/bash
# Round 4: where the region-set encode spends its time (BFHIP_SETS_STOP), and the conditional-
# subtraction modulo (BFHIP_MOD_SUB) on the P = 8 step and the north-star step.
export TMPDIR=/tmp
TAG=${1:-r04e}
# parity first: the modulo and route changes touch every offset
timeout -k 10 560 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_digests.py tests/test_gpu_region_sets.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_${TAG}_parity.log 2>&1 || exit $?
for st in 0 1 2 3; do
    BFHIP_SETS_STOP=$st timeout -k 10 200 python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --steps 3 \
        > gpurun_out/sim_sets_stop${st}_${TAG}.json 2>/dev/null || exit $?
    (echo -n "{\"stop\": $st, \"line\": "; cat gpurun_out/sim_sets_stop${st}_${TAG}.json; echo "}") >> gpurun_out/sim_sets_stop_${TAG}.jsonl
done
for ms in 1 0 1 0; do
    BFHIP_MOD_SUB=$ms timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 \
        > gpurun_out/sim_P8_modsub${ms}_${TAG}.json 2>/dev/null || exit $?
    (echo -n "{\"mod_sub\": $ms, \"line\": "; cat gpurun_out/sim_P8_modsub${ms}_${TAG}.json; echo "}") >> gpurun_out/sim_P8_modsub_${TAG}.jsonl
    BFHIP_MOD_SUB=$ms timeout -k 10 150 python bench.py --steps 10 --warmup 3 --no-secondary --no-cpu-baseline \
        --no-host-api --no-reference-shapes > gpurun_out/bench_modsub${ms}_${TAG}.json 2>/dev/null || exit $?
    (echo -n "{\"mod_sub\": $ms, \"line\": "; cat gpurun_out/bench_modsub${ms}_${TAG}.json; echo "}") >> gpurun_out/bench_modsub_${TAG}.jsonl
done

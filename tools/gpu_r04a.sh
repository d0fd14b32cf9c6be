#!/bin/bash
# Round 4, first pass: the region-set tests alone (new kernels), the replicated sims, the
# 10B apply's XCD grouping A/B and the driver's bench.  A fault, abort or time limit in any
# step ends the script (no further GPU work).
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_region_sets.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_r04a_sets.log 2>&1
rc=$?
case $rc in 0|1) ;; *) echo "region-set tests ended with $rc: stopping"; exit $rc ;; esac
bash tools/gpu_round.sh r04a repl || exit $?
for xg in 1 2 4 1 2 4; do
    BFHIP_APPLY_XG=$xg timeout -k 10 150 python bench.py --config 10b --steps 10 --warmup 3 --no-secondary \
        --no-cpu-baseline --no-host-api --no-reference-shapes > gpurun_out/ab_xg${xg}_r04a.json 2>/dev/null || exit $?
    (echo -n "{\"xg\": $xg, \"line\": "; cat gpurun_out/ab_xg${xg}_r04a.json; echo "}") >> gpurun_out/ab_xg_r04a.jsonl
done
for cfg in nstar 10b; do
    for d in 1 2 1 2; do
        BFHIP_MID_DEPTH=$d timeout -k 10 150 python bench.py --config $cfg --steps 10 --warmup 3 --no-secondary \
            --no-cpu-baseline --no-host-api --no-reference-shapes > gpurun_out/ab_mid_r04a.json 2>/dev/null || exit $?
        (echo -n "{\"depth\": $d, \"line\": "; cat gpurun_out/ab_mid_r04a.json; echo "}") >> gpurun_out/ab_mid_r04a.jsonl
    done
done
bash tools/gpu_round.sh r04a bench

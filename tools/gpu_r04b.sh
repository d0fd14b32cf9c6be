#!/bin/bash
# Round 4, second pass: region-set tests, the replicated sims (kernel trace of the sets form),
# the full GPU suite with per-test durations, smoke().  A fault, abort or time limit ends it.
export TMPDIR=/tmp
TAG=${1:-r04b}
timeout -k 10 240 python -u -m pytest tests/test_gpu_region_sets.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_${TAG}_sets.log 2>&1
rc=$?
case $rc in 0|1) ;; *) echo "region-set tests ended with $rc: stopping"; exit $rc ;; esac
bash tools/gpu_round.sh $TAG repl || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sets_${TAG} -o run -- \
    python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --fused-hash --steps 3 \
    > gpurun_out/prof_sets_${TAG}.json 2>/dev/null || exit $?
PYTEST_EXTRA="--durations=100" bash tools/gpu_round.sh $TAG tests smoke

#!/bin/bash
# Round 4: region-set tests and the replicated sims after the encode rework.
export TMPDIR=/tmp
TAG=${1:-r04d}
timeout -k 10 240 python -u -m pytest tests/test_gpu_region_sets.py tests/test_gpu_dist_gloo.py -k "sets or replicated" \
    -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_${TAG}_sets.log 2>&1
rc=$?
case $rc in 0|1) ;; *) echo "region-set tests ended with $rc: stopping"; exit $rc ;; esac
bash tools/gpu_round.sh $TAG repl || exit $?

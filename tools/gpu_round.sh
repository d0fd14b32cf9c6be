#!/bin/bash
# Full GPU-box pass: every -m gpu test, smoke(), the default bench line, a
# kernel-trace profile of the bench, and the PMC passes (tools/pmc_passes.sh).
# Run from the repo root: gpurun -- bash tools/gpu_round.sh <tag>
export TMPDIR=/tmp
TAG=${1:-round}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api \
    > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err &&
bash tools/pmc_passes.sh

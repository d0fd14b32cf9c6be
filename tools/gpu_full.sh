#!/bin/bash
# Full GPU pass: every -m gpu test, smoke(), the driver's bench command, a kernel-trace profile
# of it.  gpurun -- bash tools/gpu_full.sh <tag>
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/tests_${TAG}.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes \
    > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || exit 1

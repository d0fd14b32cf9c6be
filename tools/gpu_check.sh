#!/bin/bash
# GPU-box check: parity tests selected by $1 (pytest -k expression, "all" for the
# whole -m gpu suite), then the north-star bench under a kernel-trace profile.
# Run from the repo root: gpurun -- bash tools/gpu_check.sh '<expr>' [tag]
export TMPDIR=/tmp
SEL=${1:-all}
TAG=${2:-check}
if [ "$SEL" = "all" ]; then KOPT=(); else KOPT=(-k "$SEL"); fi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KOPT[@]}" \
    > gpurun_out/tests_${TAG}.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes \
    > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err

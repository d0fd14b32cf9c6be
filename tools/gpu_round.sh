#!/bin/bash
# Full GPU-box pass: every -m gpu test, smoke(), the driver's bench command, a kernel-trace
# profile of the bench, and the PMC passes (tools/pmc_passes.sh).
# Run from the repo root: gpurun -- bash tools/gpu_round.sh <tag> [steps...]
#   steps: tests smoke bench prof pmc (default: all)
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
    esac || { echo "step $st failed: $?"; exit 1; }
done

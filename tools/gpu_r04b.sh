#!/bin/bash
# Round 4, second pass: the full GPU suite with per-test durations, then smoke().
export TMPDIR=/tmp
PYTEST_EXTRA="--durations=100" bash tools/gpu_round.sh ${1:-r04b} tests smoke

#!/bin/bash
# Build A/B variants of libbfhip.so (on the CPU host, before gpurun):
#   ab_libs/<name>/libbfhip.so built with the given -D flags; select one with BFHIP_LIB=...
set -e
cd "$(dirname "$0")/.."
# Variants: NAME=FLAGS pairs, e.g. bash tools/build_ab_libs.sh v1=-DMY_KNOB=1 (the r01 knobs are folded in).
# The environment A/B knobs of DESIGN §6f (BFHIP_APPLY_*, BFHIP_SETS_*, BFHIP_L2_*, ...) are
# compiled only with -DBFHIP_AB_KNOBS: bash tools/build_ab_libs.sh ab=-DBFHIP_AB_KNOBS
for nv in "$@"; do
    for pair in $nv; do
        make -s -j8 -C redis-bloomfilter_amd/csrc OUTDIR=$PWD/ab_libs/${pair%%=*} EXTRA="${pair#*=}"
    done
done

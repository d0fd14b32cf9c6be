#!/bin/bash
# Build A/B variants of libbfhip.so (on the CPU host, before gpurun):
#   ab_libs/<name>/libbfhip.so built with the given -D flags; select one with BFHIP_LIB=...
set -e
cd "$(dirname "$0")/.."
# Variants: NAME=FLAGS pairs, e.g. bash tools/build_ab_libs.sh pl1=-DBF_PROBE_LOAD=1 short0=-DBF_SHA1_SHORT=0
for nv in "${@:-pl1=-DBF_PROBE_LOAD=1 pl2=-DBF_PROBE_LOAD=2}"; do
    for pair in $nv; do
        make -s -j8 -C redis-bloomfilter_amd/csrc OUTDIR=$PWD/ab_libs/${pair%%=*} EXTRA="${pair#*=}"
    done
done

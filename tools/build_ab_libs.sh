#!/bin/bash
# Build include? probe-load A/B variants of libbfhip.so (on the CPU host, before gpurun):
#   ab_libs/pl<N>/libbfhip.so with -DBF_PROBE_LOAD=<N>; select one with BFHIP_LIB=...
set -e
cd "$(dirname "$0")/.."
for v in 1 2; do
    make -s -j8 -C redis-bloomfilter_amd/csrc OUTDIR=$PWD/ab_libs/pl$v EXTRA=-DBF_PROBE_LOAD=$v
done

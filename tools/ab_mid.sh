#!/bin/bash
# bin_mid bucket-count A/B (ab_libs/m{128,256,512}): north-star bench twice interleaved, then the
# P = 8 per-rank simulation per variant.  Record of the r02x A/B
# (profiles/ab_r02/mid_buckets_128_256_512.jsonl): the variants were built with
# tools/build_ab_libs.sh m256=-DBF_MID_BUCKETS=256 ... while kMidBuckets took that macro; the
# knob was folded out afterwards (128 kept), so rerunning needs it restored in bf_binned.hip.
export TMPDIR=/tmp
L=ab_libs
bash tools/ab_bench.sh mid "BFHIP_LIB=$L/m128/libbfhip.so" "BFHIP_LIB=$L/m256/libbfhip.so" "BFHIP_LIB=$L/m512/libbfhip.so" \
    "BFHIP_LIB=$L/m128/libbfhip.so" "BFHIP_LIB=$L/m256/libbfhip.so" "BFHIP_LIB=$L/m512/libbfhip.so" || exit 1
for v in m128 m256 m512; do
    BFHIP_LIB=$L/$v/libbfhip.so timeout -k 10 120 python tools/sim_rank.py --shards 8 --sync-free --steps 5 \
        > gpurun_out/sim_mid_$v.json 2> gpurun_out/sim_mid_$v.err || exit 1
done

#!/bin/bash
# r02 counters where hashing or sparsity dominates: VALU and traffic
# passes for the 1M@1 % filter driven with 2^24-key batches (1m_big) and for 10B@0.01 %
# (10b), plus kernel traces of both.  Run from the repo root on the GPU box.
export TMPDIR=/tmp
for cfg in 1m_big 10b; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02_${cfg} -o run -- \
        python bench.py --config $cfg --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes \
        > gpurun_out/bench_prof_r02_${cfg}.json 2> gpurun_out/bench_prof_r02_${cfg}.err || exit 1
    bash tools/pmc_passes.sh $cfg r02_${cfg} valu rd wr || exit 1
done

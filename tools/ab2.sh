# A/B of library builds: the in-tree libbfhip.so vs variants under lib/variants/.
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
timeout -k 10 120 $B > gpurun_out/ab_base.json 2>/dev/null &&
for v in redis-bloomfilter_amd/lib/variants/*.so; do
    BFHIP_LIB=$PWD/$v timeout -k 10 120 $B > gpurun_out/ab_$(basename $v .so).json 2>/dev/null || exit 1
done

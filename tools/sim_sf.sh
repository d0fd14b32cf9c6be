export TMPDIR=/tmp
for P in 8 4; do
  timeout -k 10 120 python tools/sim_rank.py --shards $P --sync-free --steps 5 > gpurun_out/sim_sf_P$P.json 2> gpurun_out/sim_sf_P$P.err || exit 1
done

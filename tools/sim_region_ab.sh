export TMPDIR=/tmp
for r in 19 18 19 18; do
  BFHIP_BIN_REGION_LOG2=$r timeout -k 10 120 python tools/sim_rank.py --shards 8 --sync-free --steps 5 >> gpurun_out/sim_reg.jsonl 2>> gpurun_out/sim_reg.err || exit 1
done

#!/bin/bash
# GPU-box passes, one script for every round (no per-round one-off scripts).
# Run from the repo root: gpurun -- bash tools/gpu_round.sh <tag> [steps...]
#   tests      every -m gpu test (PYTEST_EXTRA adds flags, e.g. --durations=100)
#   parity     the parity files alone: parity, distributed primitives, digests, region sets
#   sets       region-set tests + the replicated / region-set multi-rank gloo cases
#   edge       the forced-binned edge cases at every region size (test_binned_edge_cases)
#   lua        the Lua layout's GPU tests (host and device entry points)
#   seq        every test file that reaches the sequential per-key flags (bf_seq.hip)
#   benchlua   the lua_1m secondary alone (bench.py --config 10k --secondary lua_1m)
#   smoke      __graft_entry__.smoke()
#   bench      the driver's bench command (--gpus 1 --steps 20 --warmup 5)
#   bench10b / bench200b / bench100m   the other single-GPU configs
#   prof       kernel trace (rocprofv3 --kernel-trace --stats) of a short bench run
#   pmc        the PMC passes of tools/pmc_passes.sh on the north-star bench
#   pmcstall   the stall / LDS pass of the per-rank models (PMC_WORKLOADS)
#   pmcsum     the PMC summaries made on the box (gpurun_out/pmcsum/), raw counter files deleted
#   pmcsec     the same passes for every secondary workload and per-rank model (PMC_WORKLOADS,
#              default 1m 1m_big 100m 10b 200b lua_1m model_P8_nstar model_P8_200b model_repl8_10b); then
#              python tools/pmc_finalize.py <tag> on the CPU host writes profiles/pmc_<tag>_*.json
#   simP8      the P = 8 per-rank step (tools/sim_rank.py): time + stall/LDS + VALU counters
#   simP8t     the P = 8 per-rank step, time only (SIMCFG=200b: BASELINE configs[4]'s filter)
#   repl       one replica's step of the replicated 10B x 8 and north-star x 2 layouts, per
#              insert form
#   replovl    the region-set replica steps, plain vs the next encode on a second stream (interleaved)
#   replprof   kernel trace of the 10B x 8 region-set replica step
#   replpmc    stall/LDS + VALU counters of the 10B x 8 region-set replica step
#   ablib      one command (AB_CMD) over A/B libraries built side by side on the box from AB_BUILD
#              ("name=-DFLAGS ...", tools/build_ab_libs.sh; ab_libs/ is gpurun-ignored): AB_LIBS names ab_libs/<name>
#              (interleaved, e.g. "old ab old ab"); lines appended to gpurun_out/ablib_<tag>.jsonl
#   ab         an A/B over one environment variable: AB_VAR, AB_VALUES (interleaved, e.g.
#              "1 0 1 0"), AB_CMD in {nstar, 10b, 200b, simP8, simP4, simP8_200b, repl10b, replnstar,
#              repl10bf, replnstarf (the fused-hash region-set steps), repl10bo (... with the next
#              encode on a second stream)}; lines appended to
#              gpurun_out/ab_${AB_VAR}_<tag>.jsonl.  The shipped library reads no A/B knob: the step
#              loads AB_LIB (default ab_libs/ab/libbfhip.so, built on the box by
#              `bash tools/build_ab_libs.sh ${AB_BUILD:-ab=-DBFHIP_AB_KNOBS}` when absent)
# Default: tests smoke bench prof pmc.  Every GPU step runs under its own time limit; a failing
# step ends the script (no further GPU work after a fault, abort or time limit).
export TMPDIR=/tmp
TAG=${1:-round}
shift
STEPS=${*:-tests smoke bench prof pmc}
NOEXTRA="--no-secondary --no-cpu-baseline --no-host-api --no-reference-shapes"
STALL="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
VALU="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_SALU"
SIMCFG=${SIMCFG:-nstar}                       # simP8 / simP8t: the filter (nstar, 200b)
SIMSFX=$([ "$SIMCFG" = nstar ] || echo "_$SIMCFG")
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"

ab_cmd() {   # one A/B line's command, stdout = its JSON
    case $1 in
        nstar|10b|200b) timeout -k 10 150 python bench.py --config $1 --steps 10 --warmup 3 $NOEXTRA 2>>"$ABERR" ;;
        simP8)   timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 2>>"$ABERR" ;;
        simP4)   timeout -k 10 120 python tools/sim_rank.py --shards 4 --chunks --steps 5 2>>"$ABERR" ;;
        simP8_200b) timeout -k 10 180 python tools/sim_rank.py --config 200b --shards 8 --chunks --steps 5 2>>"$ABERR" ;;
        repl10b) timeout -k 10 200 python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --steps 3 2>>"$ABERR" ;;
        replnstar) timeout -k 10 120 python tools/sim_rank.py --replicated 2 --config nstar --gathered sets --steps 5 2>>"$ABERR" ;;
        repl10bf) timeout -k 10 200 python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --fused-hash \
                      --steps 3 2>>"$ABERR" ;;
        replnstarf) timeout -k 10 120 python tools/sim_rank.py --replicated 2 --config nstar --gathered sets --fused-hash \
                      --steps 5 2>>"$ABERR" ;;
        simP8digside) timeout -k 10 120 python tools/sim_rank.py --shards 8 --chunks --steps 5 --dig --dig-side \
                      --no-hash-split 2>>"$ABERR" ;;
        repl10bo) timeout -k 10 200 python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --fused-hash \
                      --overlap-encode apply --steps 3 2>>"$ABERR" ;;
        *) echo "unknown AB_CMD $1" >&2; return 2 ;;
    esac
}

for st in $STEPS; do
    case $st in
        tests)  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
                    ${PYTEST_EXTRA:-} > gpurun_out/tests_${TAG}.log 2>&1 ;;
        parity) timeout -k 10 560 $PYT tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_digests.py \
                    tests/test_gpu_region_sets.py > gpurun_out/tests_${TAG}_parity.log 2>&1 ;;
        sets)   timeout -k 10 700 $PYT tests/test_gpu_region_sets.py tests/test_gpu_dist_gloo.py -k "sets or replicated" \
                    > gpurun_out/tests_${TAG}_sets.log 2>&1 ;;
        edge)   timeout -k 10 500 $PYT tests/test_gpu_parity.py -k binned_edge \
                    > gpurun_out/tests_${TAG}_edge.log 2>&1 ;;
        lua)    timeout -k 10 300 $PYT tests/test_gpu_lua.py > gpurun_out/tests_${TAG}_lua.log 2>&1 ;;
        seq)    timeout -k 10 500 $PYT tests/test_gpu_lua.py tests/test_gpu_parity.py tests/test_gpu_per_key.py \
                    tests/test_gpu_dirty_sync.py tests/test_gpu_engines.py tests/test_gpu_multi.py \
                    tests/test_gpu_reference_shapes.py > gpurun_out/tests_${TAG}_seq.log 2>&1 ;;
        benchlua) timeout -k 10 200 python bench.py --config 10k --secondary lua_1m --models none --steps 5 --warmup 2 \
                    --no-cpu-baseline --no-host-api --no-reference-shapes \
                    > gpurun_out/bench_lua_${TAG}.json 2> gpurun_out/bench_lua_${TAG}.err ;;
        smoke)  timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_${TAG}.log 2>&1 ;;
        bench)  timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 \
                    > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err ;;
        bench10b|bench200b|bench100m)
                timeout -k 10 300 python bench.py --config ${st#bench} --steps 20 --warmup 5 $NOEXTRA \
                    > gpurun_out/bench_${st#bench}_${TAG}.json 2> gpurun_out/bench_${st#bench}_${TAG}.err ;;
        prof)   timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
                    python bench.py --steps 5 --warmup 2 $NOEXTRA \
                    > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err ;;
        pmc)    bash tools/pmc_passes.sh nstar ${TAG}_nstar ;;
        pmcsec) for w in ${PMC_WORKLOADS:-1m 1m_big 100m 10b 200b lua_1m model_P8_nstar model_P8_200b model_repl8_10b}; do
                    bash tools/pmc_passes.sh $w ${TAG}_$w || exit 1
                done ;;
        pmcsum) python tools/pmc_finalize.py ${TAG} --box > gpurun_out/pmcsum_${TAG}.log 2>&1 ;;   # (on the box:
                # summaries to gpurun_out/pmcsum/, raw CSVs deleted so the call's output comes back)
        pmcstall)   # the stall / LDS pass of the per-rank models (VERDICT r05 item 1's counters)
                for w in ${PMC_WORKLOADS:-model_P8_200b model_P8_nstar model_repl8_10b}; do
                    bash tools/pmc_passes.sh $w ${TAG}_$w stall || exit 1
                done ;;
        simP8t) timeout -k 10 180 python tools/sim_rank.py --config $SIMCFG --shards 8 --chunks --steps 5 \
                    > gpurun_out/sim_P8${SIMSFX}_${TAG}.json 2> gpurun_out/sim_P8${SIMSFX}_${TAG}.err ;;
        simP8)  timeout -k 10 180 python tools/sim_rank.py --config $SIMCFG --shards 8 --chunks --steps 5 \
                    > gpurun_out/sim_P8${SIMSFX}_${TAG}.json 2> gpurun_out/sim_P8${SIMSFX}_${TAG}.err &&
                timeout -s KILL 150 rocprofv3 --pmc $STALL --output-format csv \
                    -d gpurun_out/pmc_${TAG}_P8${SIMSFX}_stall -o run -- python tools/sim_rank.py --config $SIMCFG \
                    --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_P8${SIMSFX}_stall.log 2>&1 &&
                timeout -s KILL 150 rocprofv3 --pmc $VALU --output-format csv \
                    -d gpurun_out/pmc_${TAG}_P8${SIMSFX}_valu -o run -- python tools/sim_rank.py --config $SIMCFG \
                    --shards 8 --chunks --steps 2 > gpurun_out/pmc_${TAG}_P8${SIMSFX}_valu.log 2>&1 ;;
        repl)   for g in digests sets "sets --fused-hash"; do
                    timeout -k 10 240 python tools/sim_rank.py --replicated 8 --config 10b --gathered $g --steps 3 \
                        >> gpurun_out/sim_repl_${TAG}.jsonl 2>> gpurun_out/sim_repl_${TAG}.err || exit 1
                done &&
                for g in keys sets "sets --fused-hash"; do
                    timeout -k 10 120 python tools/sim_rank.py --replicated 2 --config nstar --gathered $g --steps 5 \
                        >> gpurun_out/sim_repl_${TAG}.jsonl 2>> gpurun_out/sim_repl_${TAG}.err || exit 1
                done ;;
        replovl)   # the region-set replica step with the next encode beside the apply + include? (sim_rank --overlap-encode)
                for o in "" "--overlap-encode apply" "--overlap-encode include" "" "--overlap-encode apply" "--overlap-encode include"; do
                    timeout -k 10 240 python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --fused-hash $o \
                        --steps 3 >> gpurun_out/sim_replovl_${TAG}.jsonl 2>> gpurun_out/sim_replovl_${TAG}.err &&
                    timeout -k 10 120 python tools/sim_rank.py --replicated 2 --config nstar --gathered sets --fused-hash $o \
                        --steps 5 >> gpurun_out/sim_replovl_${TAG}.jsonl 2>> gpurun_out/sim_replovl_${TAG}.err || exit 1
                done ;;
        replprof)
                timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sets_${TAG} -o run -- \
                    python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --fused-hash --steps 3 \
                    > gpurun_out/prof_sets_${TAG}.json 2>/dev/null ;;
        replpmc)
                timeout -s KILL 150 rocprofv3 --pmc $STALL --output-format csv -d gpurun_out/pmc_${TAG}_sets_1 -o run -- \
                    python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --steps 1 \
                    > gpurun_out/pmc_${TAG}_sets_1.log 2>&1 &&
                timeout -s KILL 150 rocprofv3 --pmc $VALU --output-format csv -d gpurun_out/pmc_${TAG}_sets_2 -o run -- \
                    python tools/sim_rank.py --replicated 8 --config 10b --gathered sets --steps 1 \
                    > gpurun_out/pmc_${TAG}_sets_2.log 2>&1 ;;
        ab)     ABERR=gpurun_out/ab_${AB_VAR}_${TAG}.err
                export BFHIP_LIB=${AB_LIB:-$PWD/ab_libs/ab/libbfhip.so}
                # ab_libs/ is gpurun-ignored (A/B builds never ship beside the product): build on the box
                [ -f "$BFHIP_LIB" ] || timeout -k 10 600 bash tools/build_ab_libs.sh ${AB_BUILD:-ab=-DBFHIP_AB_KNOBS} \
                    > gpurun_out/ab_build_${TAG}.log 2>&1 || exit 2
                [ -f "$BFHIP_LIB" ] || { echo "no A/B library $BFHIP_LIB"; exit 2; }
                for v in ${AB_VALUES:?}; do
                    line=$(export "${AB_VAR:?}=$v"; ab_cmd "${AB_CMD:?}") || exit $?
                    echo "{\"var\": \"$AB_VAR\", \"value\": \"$v\", \"cmd\": \"$AB_CMD\", \"line\": $line}" \
                        >> gpurun_out/ab_${AB_VAR}_${TAG}.jsonl
                done ;;
        ablib)  ABERR=gpurun_out/ablib_${TAG}.err   # the same command over A/B libraries (ab_libs/<name>)
                # built on the box from AB_BUILD ("name=-DFLAGS ..."; ab_libs/ does not travel)
                [ -z "${AB_BUILD:-}" ] || timeout -k 10 900 bash tools/build_ab_libs.sh $AB_BUILD \
                    > gpurun_out/ablib_build_${TAG}.log 2>&1 || exit 2
                for lib in ${AB_LIBS:?}; do
                    [ -f ab_libs/$lib/libbfhip.so ] || { echo "no A/B library ab_libs/$lib"; exit 2; }
                    line=$(export BFHIP_LIB=$PWD/ab_libs/$lib/libbfhip.so; ab_cmd "${AB_CMD:?}") || exit $?
                    echo "{\"lib\": \"$lib\", \"cmd\": \"$AB_CMD\", \"line\": $line}" >> gpurun_out/ablib_${TAG}.jsonl
                done ;;
        *)      echo "unknown step $st"; exit 2 ;;
    esac || { echo "step $st failed: $?"; exit 1; }
done

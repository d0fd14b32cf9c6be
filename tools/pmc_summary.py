#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per hot kernel.

    python tools/pmc_summary.py gpurun_out/pmc_* [--batch 16777216] [--json out.json]

Keeps the bench's launches of the hot kernels — the direct include? / insert
kernels (bf_keys_kernel<1|2|3>, only launches over a full batch: Grid_Size ==
batch) and the binned insert pipeline's kernels — averages each counter per
launch, and derives HBM bytes per launch with the gfx950 correction (read
requests weighted 128/64/32 B by TCC_EA0_RDREQ_128B / _64B / _32B; write
requests 64/32 B by TCC_EA0_WRREQ_64B).  Keys of the output are the kernel
names bench.py's bf_profile timing uses.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

KERNELS = {
    "bf_keys_kernel<INCLUDE>": re.compile(r"bf_keys_kernel<1>"),
    "bf_keys_kernel<INSERT>": re.compile(r"bf_keys_kernel<2>"),
    "bf_keys_kernel<INSERT_FLAGS>": re.compile(r"bf_keys_kernel<3>"),
    "bf_include_hash_kernel": re.compile(r"bf_include_hash_kernel"),
    "bf_keys_kernel<HASH>": re.compile(r"bf_keys_kernel<5>"),
    "digest_kernel<INCLUDE>": re.compile(r"bf_digest_kernel<1>"),
    "digest_kernel<INSERT>": re.compile(r"bf_digest_kernel<[23]>"),   # (3: INSERT_FLAGS, any_new asked)
    "bin_front": re.compile(r"bin_front_kernel<false>"),
    "bin_front_digest": re.compile(r"bin_front_kernel<true>"),
    "bin_front_wide": re.compile(r"bin_front_wide_(dig_)?kernel"),
    "bin_mid": re.compile(r"bin_mid_kernel"),
    "bin_apply": re.compile(r"bin_apply_(pipe_)?kernel"),
    "bin_test": re.compile(r"bin_test_kernel"),
    # the Lua layout (bf_lua.hip, bench.py lua_config)
    "lua_check": re.compile(r"lua_check_kernel"),
    "lua_seq_candidates": re.compile(r"seq_candidates_kernel|seq_bin_count_kernel|seq_bin_place_kernel"),
    "lua_seq_mark": re.compile(r"seq_mark_kernel|seq_region_kernel"),
    # the per-rank models (tools/sim_rank.py: bench.py's multi_gpu_models legs), named as their
    # bf_profile marks
    "route_chunks_dig": re.compile(r"route_chunks_idx_kernel<false|route_front32_kernel<false, true, true, true>"),
    "route_chunks_slot_dig": re.compile(r"route_chunks_idx_kernel<true|route_front32_kernel<true, true, true, true>"),
    "chunk_group": re.compile(r"chunk_group_sum_kernel"),
    "mid_chunks": re.compile(r"bin_mid_chunks_kernel<false"),
    "mid_chunks_keys": re.compile(r"bin_mid_chunks_kernel<true"),
    "apply_test": re.compile(r"bin_apply_test_kernel"),
    "unsort_packed": re.compile(r"chunk_unsort_kernel"),
    "test_l2": re.compile(r"chunk_test_l2_kernel"),
    "pack_answers": re.compile(r"pack_segments_kernel"),
    "combine_chunks": re.compile(r"combine_chunks_packed_kernel"),
    "sets_encode": re.compile(r"sets_encode_kernel"),
    "sets_encode_persistent": re.compile(r"sets_encode_persistent_kernel"),   # (an encoder handle's)
    "sets_apply": re.compile(r"sets_apply_kernel"),
}
FULL_BATCH = ("bf_keys_kernel", "digest_kernel")   # grid = one lane per key: keep full-batch launches only


def load(dirs, batch):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(path)):
                for name, rx in KERNELS.items():
                    if rx.search(r["Kernel_Name"]):
                        if name.startswith(FULL_BATCH) and int(r["Grid_Size"]) != batch:
                            continue
                        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                        key = (path, r["Dispatch_Id"])
                        if key not in seen:
                            seen.add(key)
                            dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return acc, dur


def derive(c):
    g = lambda n: (sum(c[n]) / len(c[n])) if c.get(n) else None  # noqa: E731
    out = {k: g(k) for k in sorted(c)}
    rd, rd32, bub = g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_RDREQ_32B_sum"), g("TCC_BUBBLE_sum")
    if rd is not None and rd32 is not None and bub is not None:
        # rocprofv3's FETCH_SIZE expression: on gfx950 it tallies 128-B requests at 64 B
        # (MI355X_MICROARCH.md §HBM), kept for comparison only.
        out["read_bytes_fetch_size_formula"] = bub * 128 + (rd - bub - rd32) * 64 + rd32 * 32
    r128, r64 = g("TCC_EA0_RDREQ_128B_sum"), g("TCC_EA0_RDREQ_64B_sum")
    if r128 is not None and r64 is not None and rd32 is not None:
        # gfx950 correction: weight each request by the size the fabric actually moved.
        out["read_bytes"] = r128 * 128 + r64 * 64 + rd32 * 32
    wr, wr64 = g("TCC_EA0_WRREQ_sum"), g("TCC_EA0_WRREQ_64B_sum")
    if wr is not None and wr64 is not None:
        out["write_bytes"] = (wr - wr64) * 32 + wr64 * 64   # atomics are counted here (32 B each)
    if g("FETCH_SIZE") is not None:
        out["FETCH_SIZE_bytes"] = g("FETCH_SIZE") * 1024
    if g("WRITE_SIZE") is not None:
        out["WRITE_SIZE_bytes"] = g("WRITE_SIZE") * 1024
    # VALU (the hash-bound kernels): SQ_ACTIVE_INST_VALU counts quad-cycles (MI355X_MICROARCH.md
    # per-instruction table), summed over every SIMD; GRBM_GUI_ACTIVE is summed over the 8 XCDs,
    # so the kernel's cycles are GRBM_GUI_ACTIVE / 8.  valu_busy = the fraction of the 1024
    # SIMDs' cycles spent issuing VALU instructions.
    av, gui = g("SQ_ACTIVE_INST_VALU"), g("GRBM_GUI_ACTIVE")
    if av is not None and gui:
        out["valu_busy"] = av * 4 / (1024 * gui / 8)
    if g("SQ_INSTS_VALU") is not None and g("SQ_BUSY_CYCLES") is not None:
        out["valu_insts_per_busy_cycle"] = g("SQ_INSTS_VALU") / max(g("SQ_BUSY_CYCLES"), 1)
    # where the waves' time goes (quad-cycles, disjoint): parked at s_waitcnt / barriers,
    # stalled at issue, issuing (MI355X_MICROARCH.md PMC table)
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for nm in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if g(nm) is not None:
                out[nm.lower().replace("sq_", "frac_")] = g(nm) / wc
    if g("SQ_LDS_IDX_ACTIVE") and g("SQ_LDS_BANK_CONFLICT") is not None:
        out["lds_bank_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    tot = sum(out.get(k) or 0 for k in ("read_bytes", "write_bytes"))
    out["hbm_bytes"] = tot if tot else None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--workload", default="nstar")
    ap.add_argument("--json")
    args = ap.parse_args()
    acc, dur = load([d for d in args.dirs if os.path.isdir(d)], args.batch)
    res = {}
    for name in KERNELS:
        if name not in acc:
            continue
        d = derive(acc[name])
        d["launches_counted"] = max(len(v) for v in acc[name].values())
        d["profiled_ms_mean"] = sum(dur[name]) / len(dur[name]) if dur[name] else None
        d["keys_per_launch"] = args.batch
        d["hbm_bytes_per_launch"] = d.get("hbm_bytes")
        if d.get("SQ_INSTS_VALU") is not None:   # one lane per key: wave instructions x 64 / keys
            d["valu_lane_insts_per_key"] = d["SQ_INSTS_VALU"] * 64 / args.batch
        if d.get("hbm_bytes"):
            d["hbm_bytes_per_key"] = d["hbm_bytes"] / args.batch
            if d.get("profiled_ms_mean"):
                d["hbm_GBps_profiled"] = d["hbm_bytes"] / (d["profiled_ms_mean"] / 1e3) / 1e9
        res[name] = d
    out = {args.workload: res}
    txt = json.dumps(out, indent=1, sort_keys=True)
    print(txt)
    if args.json:
        with open(args.json, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()

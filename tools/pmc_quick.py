#!/usr/bin/env python3
"""Per-kernel stall / VALU fractions from rocprofv3 --pmc counter_collection CSVs (one pass each).

    python tools/pmc_quick.py <dir>/run_counter_collection.csv [filter ...]

Stall pass (SQ_WAVE_CYCLES ...): wait_any / wait_inst / active / wait_inst_lds over wave cycles, LDS
bank-conflict cycles over LDS active cycles.  VALU pass: VALU busy = SQ_ACTIVE_INST_VALU * 4 /
(1024 SIMDs * GRBM_GUI_ACTIVE / 8), as tools/pmc_passes.sh's summary defines it."""
import collections
import csv
import sys


def name(n: str) -> str:
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    path, filt = sys.argv[1], sys.argv[2:]
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = name(r["Kernel_Name"])
        if filt and not any(f in k for f in filt):
            continue
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[(k, r["Counter_Name"])] += 1
    out = {}
    for k, v in d.items():
        n = launches[(k, next(iter(v)))]
        row = {"launches": n}
        if "SQ_WAVE_CYCLES" in v:
            W = v["SQ_WAVE_CYCLES"]
            row.update(wait_any=v["SQ_WAIT_ANY"] / W, wait_inst=v["SQ_WAIT_INST_ANY"] / W,
                       active=v["SQ_ACTIVE_INST_ANY"] / W, wait_inst_lds=v["SQ_WAIT_INST_LDS"] / W,
                       lds_bank_conflict=v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1))
        if "SQ_INSTS_VALU" in v and v.get("GRBM_GUI_ACTIVE"):
            row.update(valu_busy=v["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * v["GRBM_GUI_ACTIVE"] / 8),
                       valu_insts_per_launch=v["SQ_INSTS_VALU"] / n, lds_insts_per_launch=v.get("SQ_INSTS_LDS", 0) / n,
                       salu_insts_per_launch=v.get("SQ_INSTS_SALU", 0) / n)
        out[k] = {a: round(b, 4) if isinstance(b, float) else b for a, b in row.items()}
    for k, row in sorted(out.items()):
        print(k, row)


if __name__ == "__main__":
    main()

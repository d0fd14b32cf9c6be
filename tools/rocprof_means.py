#!/usr/bin/env python3
"""Mean launch time per bench kernel from a rocprofv3 --kernel-trace --stats summary:

    python tools/rocprof_means.py profiles/<tag>_kernel_stats.csv --workload nstar > profiles/rocprof_means.json

Keys are the kernel names bench.py's bf_profile timing uses, so bench.py can report its
dominant kernel's roofline fraction from the profiler beside the in-bench events."""
import argparse
import csv
import json
import re

NAMES = {
    "include_hash_kernel": r"bf_include_hash_kernel",
    "bf_keys_kernel<INCLUDE>": r"bf_keys_kernel<1>",
    "bin_front_digest": r"bin_front_kernel<true>",
    "bin_front": r"bin_front_kernel<false>",
    "bin_mid": r"bin_mid_kernel",
    "bin_apply": r"bin_apply_(pipe_)?kernel",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--workload", default="nstar")
    args = ap.parse_args()
    out = {}
    for r in csv.DictReader(open(args.csv)):
        for key, rx in NAMES.items():
            if re.search(rx, r["Name"]) and key not in out:
                out[key] = float(r["AverageNs"]) / 1e6
    print(json.dumps({args.workload: out, "source": args.csv}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

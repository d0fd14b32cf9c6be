#!/usr/bin/env python3
"""PCIe-inclusive host-pointer API rate (what the Ruby FFI driver calls): insert_many /
include_many? of 2^24 pageable numpy keys into the north-star filter, REPS timed calls each
after a warm-up; prints min and median keys/s as one JSON line.  BFHIP_LIB selects a build."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pkgload  # noqa: E402

pkg = pkgload.load()
B = 1 << 24
REPS = int(os.environ.get("REPS", "8"))


def main():
    rng = np.random.default_rng(7)
    ib, io = pkg.keys.pack_decimal(rng.integers(0, 10**9, size=B))
    pb, po = pkg.keys.pack_decimal(rng.integers(0, 2 * 10**9, size=B))
    f = pkg.Filter(9585058377, 6, device=0)
    f.insert_many(ib, io)
    f.include_many(pb, po)
    res = {}
    for name, fn in (("insert", lambda: f.insert_many(ib, io)), ("include", lambda: f.include_many(pb, po))):
        ts = []
        for _ in range(REPS):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        res[name + "_keys_per_s_best"] = B / min(ts)
        res[name + "_keys_per_s_median"] = B / statistics.median(ts)
    res["lib"] = os.environ.get("BFHIP_LIB", "in-tree")
    f.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

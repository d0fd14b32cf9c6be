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
    keep = np.empty(B, np.uint8)

    def no_prefault(fn):
        def g():
            os.environ["BFHIP_NO_PREFAULT"] = "1"
            try:
                return fn()
            finally:
                del os.environ["BFHIP_NO_PREFAULT"]
        return g
    cases = (("insert", lambda: f.insert_many(ib, io)), ("include", lambda: f.include_many(pb, po)),
             # the result buffer's page faults: without the library's prefault thread, and into a
             # caller-owned buffer that is already mapped
             ("include_no_prefault", no_prefault(lambda: f.include_many(pb, po))),
             ("include_reused_out", lambda: f.include_many(pb, po, out=keep)))
    for rep in range(2):   # interleaved passes: the box's CPU share is noisy
        for name, fn in cases:
            ts = res.setdefault("_t_" + name, [])
            for _ in range(REPS // 2):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
    for name, _ in cases:
        ts = res.pop("_t_" + name)
        res[name + "_keys_per_s_best"] = B / min(ts)
        res[name + "_keys_per_s_median"] = B / statistics.median(ts)
    res["lib"] = os.environ.get("BFHIP_LIB", "in-tree")
    f.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

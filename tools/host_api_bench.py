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

    cases = (("insert", lambda: f.insert_many(ib, io)), ("include", lambda: f.include_many(pb, po)),
             # the result buffer's page faults: into a caller-owned buffer that is already mapped
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
    # what the PCIe link and the host give on this box, for the same bytes: pinned and pageable
    # H2D of 256 MiB, and one host thread's memcpy (the staging copies run on a pool of these)
    import torch
    nb = 256 << 20
    pin = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(nb, dtype=torch.uint8, device="cuda")
    page = np.ones(nb, np.uint8)
    for name, fn in (("h2d_pinned", lambda: dev.copy_(pin, non_blocking=True)),
                     ("d2h_pinned", lambda: pin.copy_(dev, non_blocking=True)),
                     ("h2d_pageable", lambda: dev.copy_(torch.from_numpy(page)))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        res["pcie_%s_GBps" % name] = 4 * nb / (time.perf_counter() - t) / 1e9
    dst = np.empty_like(page)
    np.copyto(dst, page)
    t = time.perf_counter()
    np.copyto(dst, page)
    res["host_memcpy_1thread_GBps"] = nb / (time.perf_counter() - t) / 1e9
    tot = int(io[-1]) + 4 * B   # key bytes + uint32 relative offsets per call
    res["pcie_bytes_per_key_insert"] = tot / B
    res["insert_pcie_GBps_at_best"] = res["insert_keys_per_s_best"] * tot / B / 1e9
    res["lib"] = os.environ.get("BFHIP_LIB", "in-tree")
    f.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

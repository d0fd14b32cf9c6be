#!/usr/bin/env python3
"""Measured estimate of a two-phase include? at the north-star filter.

Two-phase include?: phase 1 probes each key's first offset directly (the early exit keeps
~1 line fill per key); phase 2 sorts the survivors' remaining k-1 probes by region and
tests them from an LDS image of each region (the binned include's mid + test passes).
Its cost is estimated from kernels that exist, on the same 1.2 GB, 50 %-dense bitset:

  T_direct  the direct include? (k = 6, early exit every probe) of B keys    (today)
  T1        the direct include? with k = 1: hash + one probe per key          (phase 1)
  T2        the binned include? (BFHIP_INCLUDE_BINNED=1) of the survivors'
            share of the batch with k = 5: hash + partition + region test    (phase 2 + a hash)
  T_hash    the k = 1 offsets of those keys (hash + 8 B store): the hash that
            phase 2 would not redo (it would read phase 1's digests)

  estimate = T1 + T2 - T_hash  (+ phase 1's digest stores, ~20 B per survivor)

Prints one JSON line.  Run on the GPU: python tools/two_phase_estimate.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
B = 1 << 24
M = 9585058377
REPS = 5


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(REPS):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / REPS


def filt(k, binned_include=False):
    os.environ["BFHIP_INCLUDE_BINNED"] = "1" if binned_include else "0"
    f = pkg.Filter(M, k, device=0)
    bench.prefill_random(f, M, k, 0, host_copy=False)
    return f


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    (ikb, iko), (qkb, qko) = bench.make_batches(10**9, B, 0, 1, dev)[0]
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    res = {}
    f6 = filt(6)
    f6.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), B, stream=sp)
    res["T_direct_ms"] = timed(lambda: f6.include_many_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(), stream=sp))
    survivors = float(out.float().mean().item())   # not the phase-1 survivors; reported for context
    f6.close()
    f1 = filt(1)
    f1.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), B, stream=sp)
    res["T1_ms"] = timed(lambda: f1.include_many_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(), stream=sp))
    p1 = float(out.float().mean().item())          # phase-1 survivors (first bit set)
    n2 = int(B * p1)
    idx = torch.empty(max(n2, 1), dtype=torch.int64, device=dev)
    res["T_hash_ms"] = timed(lambda: f1.indexes_many_dev(qkb.data_ptr(), qko.data_ptr(), n2, idx.data_ptr(), stream=sp))
    f1.close()
    f5 = filt(5, binned_include=True)
    f5.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), B, stream=sp)
    f5.profile(True)
    f5.profile_read(reset=True)
    res["T2_ms"] = timed(lambda: f5.include_many_dev(qkb.data_ptr(), qko.data_ptr(), n2, out.data_ptr(), stream=sp))
    res["T2_kernels"] = {k: v[0] / v[1] for k, v in f5.profile_read(reset=True).items()}
    f5.close()
    os.environ["BFHIP_INCLUDE_BINNED"] = "0"
    res["phase1_survivor_fraction"] = p1
    res["member_fraction_of_answers"] = survivors
    res["digest_store_ms_est"] = n2 * 20 / 5.0e12 * 1e3
    res["estimate_ms"] = res["T1_ms"] + res["T2_ms"] - res["T_hash_ms"] + res["digest_store_ms_est"]
    res["verdict"] = "reject" if res["estimate_ms"] >= res["T_direct_ms"] else "worth building"
    print(json.dumps(res))


if __name__ == "__main__":
    main()

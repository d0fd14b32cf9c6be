#!/usr/bin/env python3
"""Estimate a two-phase north-star include? from existing kernels (no new code):

    python tools/probe_two_phase.py

* phase 1 proxy: the pipelined include? kernel (bf_include_hash_dev, next batch hashed in) on a
  k = 2 handle over the same bits: probes 0 and 1 of every key, exactly as the k = 6 kernel's
  first two rounds;
* phase 2 proxy: the opt-in binned include? (BFHIP_INCLUDE_BINNED=1: keyed front with the hash,
  keyed mid, region test) on a k = 6 handle, all six probes of every key;
* the baseline: the k = 6 pipelined include? kernel (the bench's include_hash).
One JSON line with each one's kernel times and the survivors a phase 1 would hand on."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402


def main():
    pkg = pkgload.load()
    n, p, batch, _ = bench.CONFIGS["nstar"]
    m = pkg.Bloomfilter.optimal_m(n, p)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    batches = bench.make_batches(n, batch, 0, 4, dev)
    out = torch.empty(batch, dtype=torch.uint8, device=dev)
    dig = torch.empty((batch, 4), dtype=torch.int32, device=dev)
    res = {"m": m, "batch": batch}

    def timed(f, fn, reps=6):
        for _ in range(2):
            fn(0)
        torch.cuda.synchronize()
        f.profile(True)
        f.profile_read(reset=True)
        for r in range(reps):
            fn(r)
        torch.cuda.synchronize()
        ks = {name: tot / cnt for name, (tot, cnt) in f.profile_read(reset=True).items()}
        f.profile(False)
        return ks

    def inc_hash(f):
        def fn(r):
            (nkb, nko), (pkb, pko) = batches[(r + 1) % 4][0], batches[r % 4][1]
            f.include_hash_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), nkb.data_ptr(), nko.data_ptr(),
                               batch, dig.data_ptr(), stream=stream)
        return fn

    for k in (6, 2):
        f = pkg.Filter(m, k, device=0)
        bench.prefill_random(f, m, k, 0, host_copy=False)
        res["inc_hash_k%d" % k] = timed(f, inc_hash(f))
        pkb, pko = batches[0][1]
        f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        got = out.cpu()
        res["survivors_k%d" % k] = float(got.float().mean())
        f.close()
    os.environ["BFHIP_INCLUDE_BINNED"] = "1"
    f = pkg.Filter(m, 6, device=0)
    bench.prefill_random(f, m, 6, 0, host_copy=False)

    def binned(r):
        pkb, pko = batches[r % 4][1]
        f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=stream)
    res["binned_k6"] = timed(f, binned)
    f.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

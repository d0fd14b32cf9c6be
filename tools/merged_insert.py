#!/usr/bin/env python3
"""The replicated step's insert forms on one GPU (north-star filter, 50 % prefilled):
two binned inserts of 2^24 keys (own batch, then the other rank's: the N = 2 gather form
without prefetch) against ONE binned insert of both batches (bench.py --comm-prefetch 1),
plus the plain include? of 2^24 keys.  Prints one JSON line of mean ms per form."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402


def main():
    pkg = pkgload.load()
    n, p, batch, _ = bench.CONFIGS["nstar"]
    m = pkg.Bloomfilter.optimal_m(n, p)
    k = pkg.Bloomfilter.optimal_k(n, m)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    f = pkg.Filter(m, k, device=0)
    bench.prefill_random(f, m, k, 0)
    bs = bench.make_batches(n, batch, 0, 6, dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    out = torch.empty(batch, dtype=torch.uint8, device=dev)

    def timed(fn, reps=4):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    (a, ao), _ = bs[0]
    (b, bo), _ = bs[1]
    # both batches as one packed batch
    cb = torch.cat([a[: int(ao[-1])], b])
    co = torch.cat([ao, bo[1:] + ao[-1]])
    two = timed(lambda: (f.insert_many_dev(a.data_ptr(), ao.data_ptr(), batch, stream=sp),
                         f.insert_many_dev(b.data_ptr(), bo.data_ptr(), batch, stream=sp)))
    one = timed(lambda: f.insert_many_dev(cb.data_ptr(), co.data_ptr(), 2 * batch, stream=sp))
    (q, qo) = bs[0][1]   # half batch-0 members (inserted above), half fresh keys
    inc = timed(lambda: f.include_many_dev(q.data_ptr(), qo.data_ptr(), batch, out.data_ptr(), stream=sp))
    print(json.dumps({"config": "nstar", "batch": batch, "two_inserts_ms": two, "one_merged_insert_ms": one,
                      "include_ms": inc, "n2_step_compute_ms": {"two_inserts": two + inc, "merged": one + inc}}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Times the include? forms on the north-star filter (1.2 GB, 50 %-dense, 2^24-key batches,
half members) to split the fused kernel's time into probing and hashing:

  include_many_dev     hash + probe (bf_keys_kernel<INCLUDE>)
  include_digests_dev  probe only, from precomputed SHA-1 words (bf_digest_kernel<INCLUDE>)
  include_hash_dev     hash + probe + the next batch's hash (the bench's pipelined kernel)
  hash_many_dev        hash only

Prints one JSON line.  Run on the GPU: python tools/include_forms.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402

pkg = pkgload.load()
B = 1 << 24
M, K = 9585058377, 6
REPS = 10


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


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    (ikb, iko), (qkb, qko) = bench.make_batches(10**9, B, 0, 1, dev)[0]
    sp = torch.cuda.current_stream().cuda_stream
    f = pkg.Filter(M, K, device=0)
    bench.prefill_random(f, M, K, 0, host_copy=False)
    f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), B, stream=sp)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    qdig = torch.empty((B, 4), dtype=torch.int32, device=dev)
    idig = torch.empty((B, 4), dtype=torch.int32, device=dev)
    f.hash_many_dev(qkb.data_ptr(), qko.data_ptr(), B, qdig.data_ptr(), stream=sp)
    res = {
        "include_many_dev_ms": timed(lambda: f.include_many_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(),
                                                                stream=sp)),
        "include_digests_dev_ms": timed(lambda: f.include_digests_dev(qdig.data_ptr(), B, out.data_ptr(), stream=sp)),
        "include_hash_dev_ms": timed(lambda: f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(),
                                                                ikb.data_ptr(), iko.data_ptr(), B, idig.data_ptr(),
                                                                stream=sp)),
        "hash_many_dev_ms": timed(lambda: f.hash_many_dev(ikb.data_ptr(), iko.data_ptr(), B, idig.data_ptr(),
                                                          stream=sp)),
    }
    res["members"] = float(out.float().mean().item())
    f.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

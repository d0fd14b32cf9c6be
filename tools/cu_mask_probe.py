#!/usr/bin/env python3
"""Can the next insert batch's SHA-1 run BESIDE the include? instead of inside it?

The fused include?+hash kernel costs ~0.25 ms more than include? alone: the side
hash's VALU work slows the probe rounds it shares the CUs with, and two plain kernels on two
streams do not overlap (each fills the chip).  Here the two streams get disjoint CU masks
(hipExtStreamCreateWithCUMask): include? on one set of CUs, hash_many on the other, started
together.  Prints one JSON line per CU split with every form's time on the north-star filter
(1.2 GB, 50 %-dense, 2^24-key batches, half members).  Run on the GPU.
"""
import ctypes
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


def hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    lib.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    return lib


def masked_stream(lib, cus):
    words = (ctypes.c_uint32 * 8)()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return s.value


def timed(fns, streams):
    """Mean ms of REPS rounds; each round starts every fn on its stream together."""
    ext = [torch.cuda.ExternalStream(s) for s in streams]
    cur = torch.cuda.current_stream()

    def round_():
        go = torch.cuda.Event()
        go.record(cur)
        for st in ext:
            st.wait_event(go)
        for fn, s in zip(fns, streams):
            fn(s)
        for st in ext:
            e = torch.cuda.Event()
            e.record(st)
            cur.wait_event(e)

    round_()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(cur)
    for _ in range(REPS):
        round_()
    ev[1].record(cur)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / REPS


def main():
    lib = hip()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    (ikb, iko), (qkb, qko) = bench.make_batches(10**9, B, 0, 1, dev)[0]
    sp = torch.cuda.current_stream().cuda_stream
    f = pkg.Filter(M, K, device=0)
    h = pkg.Filter(1 << 20, K, device=0)   # hash_many needs a handle, not this filter
    bench.prefill_random(f, M, K, 0, host_copy=False)
    f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), B, stream=sp)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    idig = torch.empty((B, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    inc = lambda s: f.include_many_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(), stream=s)  # noqa: E731
    hsh = lambda s: h.hash_many_dev(ikb.data_ptr(), iko.data_ptr(), B, idig.data_ptr(), stream=s)  # noqa: E731
    fused = lambda s: f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), B, out.data_ptr(),  # noqa: E731
                                         ikb.data_ptr(), iko.data_ptr(), B, idig.data_ptr(), stream=s)
    full = masked_stream(lib, range(ncu))
    base = {"cus": ncu, "fused_ms": timed([fused], [full]), "include_ms": timed([inc], [full]),
            "hash_ms": timed([hsh], [full])}
    print(json.dumps(base), flush=True)
    for every in (8, 6, 5, 4, 3):   # hash CUs: every `every`-th CU (spread over the XCDs)
        hc = [c for c in range(ncu) if c % every == every - 1]
        ic = [c for c in range(ncu) if c % every != every - 1]
        sa, sb = masked_stream(lib, ic), masked_stream(lib, hc)
        res = {"hash_cus": len(hc), "include_cus": len(ic),
               "include_alone_ms": timed([inc], [sa]), "hash_alone_ms": timed([hsh], [sb]),
               "together_ms": timed([inc, hsh], [sa, sb])}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

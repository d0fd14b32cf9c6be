#!/usr/bin/env python3
"""Random 4-byte reads per second vs footprint (how much the 256 MB Infinity Cache and the
L2s help the include? probe pattern).  torch's gather: one int32 load per index."""
import json

import torch

dev = torch.device("cuda", 0)
n = 1 << 26
out = {}
for mb in (16, 64, 128, 256, 512, 1200, 4800):
    words = mb * (1 << 20) // 4
    t = torch.zeros(words, dtype=torch.int32, device=dev)
    idx = torch.randint(0, words, (n,), device=dev, dtype=torch.int64)
    for _ in range(2):
        torch.gather(t, 0, idx)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        torch.gather(t, 0, idx)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    out[mb] = {"ms": round(ms, 4), "G_reads_per_s": round(n / ms / 1e6, 2)}
    del t, idx
print(json.dumps(out))

#!/usr/bin/env python3
"""Per-rank compute of the partitioned filter at P shards, simulated on ONE GPU.

    python tools/sim_rank.py [--shards 8] [--config nstar] [--steps 5]

Builds shard 0 of a P-way partitioned north-star filter (the largest shard) and runs,
per step, the kernels one rank runs at world size P: route its 2^24-key insert batch,
apply a received batch of the same size to its shard, route its include? batch, test
a received batch, combine.  The received batches are this rank's own routed probes (in
a balanced run every rank receives about as many as it sends; every owner-local offset
is valid on shard 0, the largest).  No collective runs: the all-to-all time is not in
these numbers.  Prints one JSON line with per-kernel means (bf_profile).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--config", default="nstar", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--windows", action="store_true",
                    help="route through bf_route_windows_dev (window send buffer, no gather pass); "
                         "a device copy of the windows stands in for the receive")
    ap.add_argument("--sync-free", action="store_true",
                    help="the default exchange's compute: whole windows of cap_sf entries, device-side "
                         "counts, windowed owner ops, packed answers (PartitionedFilter._sf_*); the "
                         "received windows are this rank's own (nh == 1 configs)")
    args = ap.parse_args()
    pkg = pkgload.load()
    n_items, err, batch, _ = bench.CONFIGS[args.config]
    m = pkg.Bloomfilter.optimal_m(n_items, err)
    k = pkg.Bloomfilter.optimal_k(n_items, m)
    dev = torch.device("cuda", 0)
    eng = pkg.distributed.HipEngine(m, k, args.shards, 0, 20, dev)
    f = eng.filter
    batches = bench.make_batches(n_items, batch, 0, args.steps + 1, dev)
    torch.cuda.synchronize()

    P = args.shards
    cap = batch * k // P + batch * k // (8 * P) + 4096

    nh = eng.nh   # 2^32-bit sub-range windows per owner (1 when the shard fits 2^32 bits)

    def received(send, counts):
        """Stand-in for the receive: every window's live entries, grouped by sub-range h
        (what the grouped send/recv delivers when every source routed this batch)."""
        c = counts.cpu().tolist()
        runs = []
        for h in range(nh):
            parts = [send[(s * nh + h) * cap: (s * nh + h) * cap + c[s * nh + h]] for s in range(P)]
            runs.append((h, torch.cat(parts)))
        return runs

    def step_windows(b):
        (ikb, iko), (qkb, qko) = b
        send, _, counts = eng.route_windows(ikb, iko, batch, cap, want_slot=False)
        for h, run in received(send, counts):
            eng.shard_insert_hi(run, h)
        send, slot, counts = eng.route_windows(qkb, qko, batch, cap)
        back = torch.empty(P * nh * cap, dtype=torch.uint8, device=dev)
        c = counts.cpu().tolist()
        for h, run in received(send, counts):
            bits = torch.empty(run.numel(), dtype=torch.uint8, device=dev)
            eng.shard_test_hi(run, h, bits)
            at = 0
            for s in range(P):
                w = s * nh + h
                back[w * cap: w * cap + c[w]] = bits[at: at + c[w]]
                at += c[w]
        return eng.combine_windows(back, slot, counts, cap, batch)

    def step_sf(b):
        (ikb, iko), (qkb, qko) = b
        A = 12288
        capsf = -(-min(batch * k, batch * k // P + batch * k // (8 * P) + 4096) // A) * A
        send, _, counts = eng.route_windows(ikb, iko, batch, capsf, want_slot=False)
        rmsg = torch.cat([counts.view(P, 1), torch.zeros(P, 1, dtype=torch.int64, device=dev)], 1).contiguous()
        eng.shard_insert_windows(send, capsf, P, rmsg, 0, 2, 0)
        send, slot, counts = eng.route_windows(qkb, qko, batch, capsf)
        rmsg = torch.cat([counts.view(P, 1), torch.zeros(P, 1, dtype=torch.int64, device=dev)], 1).contiguous()
        bits = torch.empty(P * capsf, dtype=torch.uint8, device=dev)
        eng.shard_test_windows(send, capsf, P, rmsg, 0, 2, 0, bits)
        cap8 = (capsf + 7) // 8
        seg = torch.tensor([[src * capsf, capsf, src * cap8] for src in range(P)], dtype=torch.int64).to(dev)
        packed = eng.pack_answers(bits, seg, capsf, P * cap8)
        return eng.combine_windows_packed(packed, slot, counts, capsf, batch)

    def step(b):
        if args.sync_free:
            assert nh == 1
            return step_sf(b)
        if args.windows:
            return step_windows(b)
        (ikb, iko), (qkb, qko) = b
        send, _, _ = eng.route(ikb, iko, batch, want_slot=False)
        eng.shard_insert(send)
        send, slot, _ = eng.route(qkb, qko, batch)
        bits = eng.shard_test(send)
        return eng.combine(bits, slot, batch)

    step(batches[0])
    torch.cuda.synchronize()
    f.profile(True)
    f.profile_read(reset=True)
    t0 = time.perf_counter()
    for b in batches[1:]:
        step(b)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    prof = f.profile_read(reset=True)
    out = {"config": args.config, "shards": args.shards, "m": m, "k": k, "batch": batch,
           "shard_bytes": f.device_bytes, "route32": bool(eng.offset_dtype == torch.int32),
           "route": "sync-free windows" if args.sync_free else ("windows" if args.windows else "contiguous"),
           "ms_per_step_compute": wall * 1e3,
           "kernels_ms_per_step": {name: ms / args.steps for name, (ms, _) in prof.items()},
           "kernels_ms_sum": sum(ms for ms, _ in prof.values()) / args.steps,
           "note": "ms_per_step_compute includes the stand-in receive copies of --windows "
                   "(the exchange's job in a real run); kernels_ms_sum does not"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

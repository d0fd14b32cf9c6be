#!/usr/bin/env python3
"""A/B the probe policies (BFHIP_INCLUDE_FIRST_ROUND, BFHIP_INSERT_TEST) in ONE
process, interleaved rounds, on fresh device batches (cdna_hip_programming.md
§5.4 rule 24).  Prints one JSON line per (config, policy) with median/min ms.

    python tools/ab_policies.py [--configs nstar,100m,1m] [--rounds 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="nstar,100m,1m")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="BFHIP_BITS_MEM=0|BFHIP_BITS_MEM=1|BFHIP_BITS_MEM=2",
                    help="'|'-separated variants, each a ','-separated list of ENV=value")
    args = ap.parse_args()
    pkg = pkgload.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    for name in args.configs.split(","):
        n, p, batch, prefill = bench.CONFIGS[name]
        m = pkg.Bloomfilter.optimal_m(n, p)
        k = pkg.Bloomfilter.optimal_k(n, m)
        base = pkg.Filter(m, k, device=0)
        if prefill == "random":
            host = bench.prefill_random(base, m, k, 0)
        else:
            host = None
        batches = bench.make_batches(n, batch, 0, args.rounds + 1, dev)
        if host is None:   # fill by inserting the first batch
            (kb, ko), _ = batches[0]
            base.insert_many_dev(kb.data_ptr(), ko.data_ptr(), batch, stream=0)
            torch.cuda.synchronize()
        ref = base.export_redis()
        variants = []
        for spec in args.variants.split("|"):
            env = dict(kv.split("=") for kv in spec.split(",") if kv)
            saved = {kk: os.environ.get(kk) for kk in env}
            os.environ.update(env)
            f = pkg.Filter(m, k, device=0)
            for kk, vv in saved.items():
                if vv is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = vv
            variants.append((spec, f))
        times = {v[0]: {"insert": [], "include": []} for v in variants}
        out = torch.empty(batch, dtype=torch.uint8, device=dev)
        answers = {}
        for r in range(1, args.rounds + 1):
            (ikb, iko), (pkb, pko) = batches[r]
            for pol, f in variants:
                f.import_redis(ref)          # same starting state for every variant
                torch.cuda.synchronize()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), batch, stream=0)
                e[1].record()
                f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=0)
                e[2].record()
                torch.cuda.synchronize()
                times[pol]["insert"].append(e[0].elapsed_time(e[1]))
                times[pol]["include"].append(e[1].elapsed_time(e[2]))
                answers.setdefault(r, []).append(out.cpu().numpy().tobytes())
        same = all(len(set(v)) == 1 for v in answers.values())
        for pol, t in times.items():
            print(json.dumps({"config": name, "m": m, "k": k, "batch": batch, "variant": pol,
                              "insert_ms_median": float(np.median(t["insert"])), "insert_ms_min": float(np.min(t["insert"])),
                              "include_ms_median": float(np.median(t["include"])), "include_ms_min": float(np.min(t["include"])),
                              "answers_identical": same}), flush=True)
        for _, f in variants:
            f.close()
        base.close()
        del batches


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-key latency breakdown of the reference's per-key API on the hip driver.

    python tools/per_key_latency.py [--iters 2000] [--size 10000]

Times, per call (microseconds, median over --iters), each layer a facade ``insert`` /
``include`` goes through: the C ABI alone (bf_insert_many / bf_include_many of one key),
the dirty-range query and range export the write-through sync adds, and the whole facade
call with and without a FakeRedis attached.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime, as in bench.py)

import pkgload  # noqa: E402


def med_us(fn, iters):
    ts = []
    for i in range(iters):
        t0 = time.perf_counter()
        fn(i)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--size", type=int, default=10000)
    args = ap.parse_args()
    pkg = pkgload.load()
    it = args.iters
    words = ["w%07d" % i for i in range(4 * it)]
    res = {"size": args.size, "iters": it}

    bf = pkg.Bloomfilter(size=args.size, error_rate=0.01, key_name="lat", driver="hip", redis=pkg.FakeRedis())
    f = bf.driver.filter
    packed = [pkg.keys.pack([w]) for w in words]
    res["abi_insert_any_new"] = med_us(lambda i: f.insert_many(*packed[i], any_new=True), it)
    res["abi_insert"] = med_us(lambda i: f.insert_many(*packed[it + i]), it)
    res["abi_include"] = med_us(lambda i: f.include_many(*packed[i]), it)
    res["keys_pack"] = med_us(lambda i: pkg.keys.pack([words[i]]), it)
    res["dirty_ranges"] = med_us(lambda i: f.dirty_ranges(clear=True), it)
    res["export_range_4k"] = med_us(lambda i: f.export_range(0, 4096), it)
    res["facade_insert_write_through"] = med_us(lambda i: bf.insert(words[2 * it + i]), it)
    res["facade_include"] = med_us(lambda i: bf.include(words[i]), it)
    bf.driver.redis = None
    res["facade_insert_no_redis"] = med_us(lambda i: bf.insert(words[3 * it + i]), it)
    bf.driver.close()
    lua = pkg.Bloomfilter(size=args.size, error_rate=0.01, key_name="latl", driver="hip-lua", redis=pkg.FakeRedis())
    res["lua_facade_insert_write_through"] = med_us(lambda i: lua.insert(words[i]), it)
    res["lua_facade_include"] = med_us(lambda i: lua.include(words[i]), it)
    lua.driver.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

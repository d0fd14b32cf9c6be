"""Does a VALU-bound pass overlap the memory-bound include? kernel?  (measurement only)

    python tools/overlap_probe.py

On the north-star filter (1B@1 %, 50 % density): times include? alone, insert alone, and
both launched together on two streams (same handle; results not checked, timing only).
Prints one JSON line."""
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
    n_items, err, batch, _ = bench.CONFIGS["nstar"]
    B = pkg.Bloomfilter
    m = B.optimal_m(n_items, err)
    k = B.optimal_k(n_items, m)
    f = pkg.Filter(m, k, device=0)
    bench.prefill_random(f, m, k, 0, host_copy=False)
    bt = bench.make_batches(n_items, batch, 0, 4, torch.device("cuda", 0))
    out = torch.empty(batch, dtype=torch.uint8, device="cuda")
    idx = torch.empty(batch * k, dtype=torch.int64, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def inc(s, i):
        (pkb, pko) = bt[i][1]
        f.include_many_dev(pkb.data_ptr(), pko.data_ptr(), batch, out.data_ptr(), stream=s.cuda_stream)

    def ins(s, i):
        (ikb, iko) = bt[i][0]
        f.insert_many_dev(ikb.data_ptr(), iko.data_ptr(), batch, stream=s.cuda_stream)

    def idxs(s, i):
        (ikb, iko) = bt[i][0]
        f.indexes_many_dev(ikb.data_ptr(), iko.data_ptr(), batch, idx.data_ptr(), stream=s.cuda_stream)

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            with torch.cuda.stream(sa):
                torch.cuda._sleep(20_000_000)   # hold the stream while the host enqueues everything
            e0.record(sa)
            sb.wait_event(e0)
            fn()
            eb = torch.cuda.Event()
            eb.record(sb)
            sa.wait_event(eb)
            e1.record(sa)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sum(ts) / len(ts)

    res = {
        "include": timed(lambda: inc(sa, 0)),
        "insert": timed(lambda: ins(sb, 1)),
        "indexes": timed(lambda: idxs(sb, 1)),
        "include_then_insert_one_stream": timed(lambda: (inc(sa, 0), ins(sa, 1))),
        "include_with_insert": timed(lambda: (inc(sa, 0), ins(sb, 1))),
        "include_with_indexes": timed(lambda: (inc(sa, 0), idxs(sb, 1))),
        "insert_then_include_two_streams": timed(lambda: (ins(sb, 1), inc(sa, 0))),
    }
    print(json.dumps(res))
    f.close()


if __name__ == "__main__":
    main()

"""Device work of one handle is ordered across streams (include/bfhip.h, StreamOrder in
bf_api.cpp): *_dev inserts issued on two torch streams with no synchronisation between
them share the handle's binned scratch and bin_apply's plain region stores, yet the final
bitset equals the oracle's for both batches, and include? answers on a third stream see
every bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev(torch, buf, offs):
    kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
    ko = torch.from_numpy(offs.view(np.int64)).cuda()
    return kb, ko


@pytest.mark.parametrize("binned", ["1", "0"])
def test_inserts_on_two_streams(pkg, oracle, monkeypatch, binned):
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    m, k = 1437758757, 10                      # 100M@0.1 %: 180 MB, binned when forced
    rng = np.random.default_rng(71)
    batches = [pkg.keys.pack_decimal(rng.integers(0, 10**12, size=400_000)) for _ in range(4)]
    dev = [_dev(torch, b, o) for b, o in batches]
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with pkg.Filter(m, k) as f:
        for i, (kb, ko) in enumerate(dev):      # alternate streams, never synchronise between
            st = (s1 if i % 2 == 0 else s2).cuda_stream
            f.insert_many_dev(kb.data_ptr(), ko.data_ptr(), len(batches[i][1]) - 1, stream=st)
        out = torch.empty(len(batches[3][1]) - 1, dtype=torch.uint8, device="cuda")
        kb, ko = dev[3]
        f.include_many_dev(kb.data_ptr(), ko.data_ptr(), out.numel(), out.data_ptr(), stream=s3.cuda_stream)
        torch.cuda.synchronize()
        got = f.export_redis()
        ans = out.cpu().numpy()
    bits = oracle.new_bitset(m, k)
    for b, o in batches:
        oracle.insert_many(bits, m, k, b, o)
    assert got == oracle.redis_string(bits)
    assert ans.all()

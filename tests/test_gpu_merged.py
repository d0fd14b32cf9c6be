"""A merged insert of several ranks' batches (the replicated layout's step, ReplicatedFilter /
tools/sim_rank.py --replicated) on the 10B@0.01 % filter: one binned pass over a batch larger
than r02's single-pass limit (~19.9M keys at k = 13 on the 6.98 GB bitset) must leave the same
bitset as the direct (test-then-atomic) insert, and every key must then answer true.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_merged_insert_one_pass_equals_direct(pkg, monkeypatch):
    import torch
    m, k = 191701167547, 13   # BASELINE configs[3]: 10B@0.01 %
    n = (1 << 25) + 12345     # 2 ranks' 2^24-key batches and a ragged tail
    rng = np.random.default_rng(0x5EED + 77)
    ib, io = pkg.keys.pack_decimal(rng.integers(0, 10**10, size=n))
    kb = torch.from_numpy(np.concatenate([ib, np.zeros(16, np.uint8)])).cuda()
    ko = torch.from_numpy(io.view(np.int64)).cuda()
    flags = torch.zeros(2, dtype=torch.int32, device="cuda")
    monkeypatch.setenv("BFHIP_INSERT_BINNED", "1")
    fb = pkg.Filter(m, k, device=0)
    plan = fb.insert_plan(n)
    assert plan["binned"]
    # one pass: the scratch holds all n*k probes (two 4-B level arrays) at once
    assert plan["scratch_bytes"] >= 2 * 4 * n * k
    fb.profile(True)
    fb.profile_read(reset=True)
    fb.insert_many_dev(kb.data_ptr(), ko.data_ptr(), n, d_any_new=flags[0:1].data_ptr())
    torch.cuda.synchronize()
    prof = fb.profile_read(reset=True)
    fb.profile(False)
    assert prof["bin_apply"][1] == 1, prof   # the bitset streamed once
    monkeypatch.setenv("BFHIP_INSERT_BINNED", "0")
    fd = pkg.Filter(m, k, device=0)
    fd.insert_many_dev(kb.data_ptr(), ko.data_ptr(), n, d_any_new=flags[1:2].data_ptr())
    torch.cuda.synchronize()
    pb, nb = fb.device_bits()
    pd, nd = fd.device_bits()
    assert nb == nd
    D = pkg.distributed
    a = D.device_bytes_view(fb)
    b = D.device_bytes_view(fd)
    assert bool(torch.equal(a, b))
    assert flags.tolist() == [1, 1]
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    fb.include_many_dev(kb.data_ptr(), ko.data_ptr(), n, out.data_ptr())
    assert bool(out.all())
    fb.close()
    fd.close()

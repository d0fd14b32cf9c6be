"""SHA-1 words as an intermediate (include/bfhip.h: bf_hash_many_dev, bf_insert_digests_dev,
bf_include_digests_dev, bf_include_hash_dev) against the oracle: the digests are the first
four big-endian words of SHA-1(key) (ruby.rb:42-47's h[0..3]), and every op on them gives
the same bitset and answers as the same op on the keys."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED + 70


def _dev(torch, buf, offs):
    kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).cuda()
    ko = torch.from_numpy(offs.view(np.int64)).cuda()
    return kb, ko


def _want_digests(buf, offs):
    out = np.zeros((len(offs) - 1, 4), np.uint32)
    for j in range(len(offs) - 1):
        d = hashlib.sha1(bytes(buf[int(offs[j]):int(offs[j + 1])])).digest()
        out[j] = np.frombuffer(d[:16], ">u4")
    return out


def _keys(pkg, rng, n, long_every=0):
    vals = [str(int(v)) for v in rng.integers(0, 10**12, size=n)]
    if long_every:   # past the single-block SHA-1 (> 55 bytes)
        vals = [v * 9 if i % long_every == 0 else v for i, v in enumerate(vals)]
    return pkg.keys.pack(vals)


@pytest.mark.parametrize("long_every", [0, 7])
def test_hash_many_matches_sha1(pkg, long_every):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(SEED)
    buf, offs = _keys(pkg, rng, 5000, long_every)
    kb, ko = _dev(torch, buf, offs)
    dig = torch.empty((5000, 4), dtype=torch.int32, device="cuda")
    with pkg.Filter(9585058, 6) as f:
        f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), 5000, dig.data_ptr(), stream=0)
        torch.cuda.synchronize()
    np.testing.assert_array_equal(dig.cpu().numpy().view(np.uint32), _want_digests(buf, offs))


@pytest.mark.parametrize("binned", ["0", "1"])
@pytest.mark.parametrize("m,k", [(9585058, 6), (9585058377, 6), (1437758757, 10), (191701167547, 13)])
def test_digest_ops_match_oracle(pkg, oracle, monkeypatch, binned, m, k):
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("BFHIP_INSERT_BINNED", binned)
    rng = np.random.default_rng(SEED + k)
    ib, io = _keys(pkg, rng, 30_000, 11)
    pb, po = _keys(pkg, rng, 10_000)
    probe = (np.concatenate([ib, pb]), np.concatenate([io, po[1:] + io[-1]]))
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    want_inc = oracle.include_many(bits, m, k, *probe)
    kb, ko = _dev(torch, ib, io)
    qb, qo = _dev(torch, *probe)
    nq = len(probe[1]) - 1
    dig = torch.empty((30_000, 4), dtype=torch.int32, device="cuda")
    qdig = torch.empty((nq, 4), dtype=torch.int32, device="cuda")
    out = torch.empty(nq, dtype=torch.uint8, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    with pkg.Filter(m, k) as f:
        f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), 30_000, dig.data_ptr(), stream=0)
        f.insert_digests_dev(dig.data_ptr(), 30_000, flag.data_ptr(), stream=0)
        f.hash_many_dev(qb.data_ptr(), qo.data_ptr(), nq, qdig.data_ptr(), stream=0)
        f.include_digests_dev(qdig.data_ptr(), nq, out.data_ptr(), stream=0)
        torch.cuda.synchronize()
        assert int(flag.item()) == 1
        assert f.export_redis() == oracle.redis_string(bits)
        np.testing.assert_array_equal(out.cpu().numpy(), want_inc)
        flag.zero_()
        f.insert_digests_dev(dig.data_ptr(), 30_000, flag.data_ptr(), stream=0)   # nothing new
        torch.cuda.synchronize()
        assert int(flag.item()) == 0


@pytest.mark.parametrize("nq,nn", [(20_000, 20_000), (20_000, 5_000), (3_000, 20_000), (0, 4_000), (4_000, 0),
                                   (1, 257)])
def test_include_hash_fused(pkg, oracle, nq, nn):
    """include? of one batch with the next batch's hash fused in: the answers are the filter's
    as it stands, the digests are the next batch's SHA-1 words, for batches of any relative
    size (workgroups past the include? batch only hash)."""
    torch = pytest.importorskip("torch")
    m, k = 9585058377, 6
    rng = np.random.default_rng(SEED + nq + nn)
    ib, io = _keys(pkg, rng, 30_000)
    qb, qo = _keys(pkg, rng, max(nq, 1), 13)
    qo = qo[: nq + 1]
    nb, no = _keys(pkg, rng, max(nn, 1), 5)
    no = no[: nn + 1]
    bits = oracle.new_bitset(m, k)
    oracle.insert_many(bits, m, k, ib, io)
    kb, ko = _dev(torch, ib, io)
    qkb, qko = _dev(torch, qb, qo)
    nkb, nko = _dev(torch, nb, no)
    out = torch.full((max(nq, 1),), 7, dtype=torch.uint8, device="cuda")
    dig = torch.zeros((max(nn, 1), 4), dtype=torch.int32, device="cuda")
    with pkg.Filter(m, k) as f:
        f.insert_many_dev(kb.data_ptr(), ko.data_ptr(), 30_000, stream=0)
        f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), nq, out.data_ptr(), nkb.data_ptr(), nko.data_ptr(), nn,
                           dig.data_ptr(), stream=0)
        torch.cuda.synchronize()
    if nq:
        np.testing.assert_array_equal(out.cpu().numpy()[:nq], oracle.include_many(bits, m, k, qb, qo))
    if nn:
        np.testing.assert_array_equal(dig.cpu().numpy().view(np.uint32)[:nn], _want_digests(nb, no))


def test_pipelined_steps_equal_plain_steps(pkg, oracle):
    """The bench's pipelined step (insert_digests(I_i), then include_hash(Q_i, I_{i+1})) gives
    the same bitset and answers as insert_many(I_i) then include_many(Q_i)."""
    torch = pytest.importorskip("torch")
    m, k = 9585058377, 6
    rng = np.random.default_rng(SEED + 1)
    batches = []
    for _ in range(4):
        ib, io = _keys(pkg, rng, 25_000)
        qb, qo = pkg.keys.pack([pkg.keys.unpack(ib, io, j).decode() for j in range(0, 25_000, 2)] +
                               [str(int(v)) for v in rng.integers(10**12, 2 * 10**12, size=12_500)])
        batches.append(((ib, io), (qb, qo)))
    dev = [(_dev(torch, *b[0]), _dev(torch, *b[1])) for b in batches]
    outs = [torch.empty(len(b[1][1]) - 1, dtype=torch.uint8, device="cuda") for b in batches]
    digs = [torch.empty((len(b[0][1]) - 1, 4), dtype=torch.int32, device="cuda") for b in batches]
    bits = oracle.new_bitset(m, k)
    with pkg.Filter(m, k) as f:
        (kb, ko), _ = dev[0]
        f.hash_many_dev(kb.data_ptr(), ko.data_ptr(), len(batches[0][0][1]) - 1, digs[0].data_ptr(), stream=0)
        for i in range(4):
            f.insert_digests_dev(digs[i].data_ptr(), len(batches[i][0][1]) - 1, stream=0)
            (_, _), (qkb, qko) = dev[i]
            nxt = dev[i + 1][0] if i + 1 < 4 else (None, None)
            nn = len(batches[i + 1][0][1]) - 1 if i + 1 < 4 else 0
            f.include_hash_dev(qkb.data_ptr(), qko.data_ptr(), outs[i].numel(), outs[i].data_ptr(),
                               nxt[0].data_ptr() if nn else 0, nxt[1].data_ptr() if nn else 0, nn,
                               digs[i + 1].data_ptr() if nn else 0, stream=0)
        torch.cuda.synchronize()
        got = f.export_redis()
    for i, ((ib, io), (qb, qo)) in enumerate(batches):
        oracle.insert_many(bits, m, k, ib, io)
        np.testing.assert_array_equal(outs[i].cpu().numpy(), oracle.include_many(bits, m, k, qb, qo))
        assert outs[i].cpu().numpy()[:12_500].all()
    assert got == oracle.redis_string(bits)

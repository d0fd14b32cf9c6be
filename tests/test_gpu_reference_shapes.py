"""The reference's own benchmark loops (bench.py ``reference_shapes``) at small sizes, checked
against the ruby driver's restatement (oracle/oracle.py RubyDriverRestatement over FakeRedis):

* benchmark/bf_10_000.rb:20-43 — per-key include? (against a visited set) then insert of W8
  words: the error count, the first error's index and the Redis string must equal what the
  ruby driver (ruby.rb:20-30, 57-63) produces on the same words, key by key;
* benchmark/bf_100_000_flat.rb — per-key and batched insert / include? of rand(items):
  every inserted key answers true;
* BASELINE configs[2] — the 100M@0.1 % filter with write-through sync (reduced batch).
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_reference_shapes_match_ruby_driver(pkg, O):
    import bench
    words_n = 2000
    res = bench.reference_shapes(pkg, per_key_ops=500, words_n=words_n, flat_items=5000, big_keys=1 << 16)

    # the ruby driver over FakeRedis on the same words (same seeded generator as the bench)
    rng = np.random.default_rng(bench.SEED)
    words = bench._w8_words(rng, words_n)
    m = O.py_optimal_m(words_n, 0.01)
    k = O.py_optimal_k(words_n, m)
    r = pkg.FakeRedis()
    ref = O.RubyDriverRestatement({"bits": m, "hashes": k, "key_name": "ref", "redis": r})
    error, first, visited = 0, 0, set()
    for i, w in enumerate(words):
        if ref.include(w) != (w in visited):
            error += 1
            if error == 1:
                first = i
        visited.add(w)
        ref.insert(w)
    want_sha1 = hashlib.sha1(r.get("ref") or b"").hexdigest()

    for drv in ("hip", "hip-lua", "hip-test"):
        got = res["bf_10_000"][drv]
        assert got["bits"] == m and got["hashes"] == k
        assert got["ops_per_s"] > 0
    hip = res["bf_10_000"]["hip"]
    assert (hip["errors"], hip["first_error_at"]) == (error, first)
    assert hip["redis_string_sha1"] == want_sha1
    # the flat shape asserts every inserted key answers true inside reference_shapes
    for drv in ("hip", "hip-lua"):
        f = res["flat"][drv]
        assert f["per_key_sample"] == 500 and f["batched_include_keys_per_s"] > 0
    s = res["100m_sync"]
    assert s["keys"] == 1 << 16 and s["redis_string_bytes"] > 0

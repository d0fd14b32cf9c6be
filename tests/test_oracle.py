"""The oracle pinned before it is trusted (CPU only).

* FIPS 180-4 SHA-1 known answers (both restatements);
* the reference spec's only exact pin: 1000 @ 0.01 -> bits 9585, hashes 6
  (spec/redis_bloomfilter_spec.rb:56-57);
* SURVEY §7 known answers and the committed golden fixtures
  (tests/golden/golden.json, from hashlib; Node-crypto cross-checked);
* the C restatement (oracle/bf_oracle.c) against the pure-Python one.
"""
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "golden.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as fh:
        return json.load(fh)


def test_fips_sha1(golden, oracle):
    for msg, want in golden["fips_sha1"].items():
        assert hashlib.sha1(msg.encode("latin1")).hexdigest() == want
        assert oracle.sha1(msg.encode("latin1")).hex() == want
    million_a = b"a" * 1_000_000
    assert oracle.sha1(million_a).hex() == "34aa973cd4c4daa4f61eeb2bdbad27316534016f"


def test_sha1_all_lengths_vs_hashlib(oracle):
    rng = np.random.default_rng(7)
    for L in range(0, 300):
        b = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert oracle.sha1(b) == hashlib.sha1(b).digest()


def test_spec_sizing_pin(O, oracle):
    """spec/redis_bloomfilter_spec.rb:52-60."""
    assert O.py_optimal_m(1000, 0.01) == 9585
    assert O.py_optimal_k(1000, 9585) == 6
    assert oracle.optimal_m(1000, 0.01) == 9585
    assert oracle.optimal_k(1000, 9585) == 6


def test_sizing_table(golden, O, oracle):
    for row in golden["sizing"]:
        assert O.py_optimal_m(row["n"], row["p"]) == row["bits"]
        assert oracle.optimal_m(row["n"], row["p"]) == row["bits"]
        assert O.py_optimal_k(row["n"], row["bits"]) == row["hashes"]
        assert oracle.optimal_k(row["n"], row["bits"]) == row["hashes"]
    # SURVEY §8 a1/a2 figures for BASELINE.json's configs
    want = {(10_000, 0.01): (95851, 6), (10**6, 0.01): (9585058, 6), (10**8, 0.001): (1437758757, 10),
            (10**9, 0.01): (9585058377, 6), (10**10, 1e-4): (191701167547, 13),
            (2 * 10**11, 1e-4): (3834023350947, 13)}
    for (n, p), (m, k) in want.items():
        assert (O.py_optimal_m(n, p), O.py_optimal_k(n, O.py_optimal_m(n, p))) == (m, k)


def test_ruby_round_and_integer_division(O):
    assert O.ruby_round(2.5) == 3 and O.ruby_round(-2.5) == -3 and O.ruby_round(0.49999) == 0
    # Integer n: floor division before the log (bloomfilter.rb:55)
    assert O.py_optimal_k(3, 5) == 1           # 5 // 3 = 1 -> round(0.69) = 1
    assert O.py_optimal_k(3.0, 5) == 1         # float: round(0.693 * 1.667 = 1.155) = 1
    assert O.py_optimal_k(2, 5) == 1           # 5 // 2 = 2 -> round(1.386) = 1
    assert O.py_optimal_k(2.0, 5) == 2         # 2.5 * 0.693 = 1.733 -> 2
    assert O.py_optimal_k(10, 3) == 1          # 0 -> bumped to 1 (bloomfilter.rb:56)


def test_survey_known_answers(O, oracle):
    cases = {("asdlol", 9585, 6): [5260, 6438, 144, 8807, 5008, 5791],
             ("foo", 95851, 7): [61181, 74832, 85954, 69596, 70715, 28527, 39649],
             (42, 9585, 6): [6198, 1190, 536, 3493, 2299, 9036],
             ("", 9585, 6): [8986, 4917, 7472, 7054, 4436, 1889]}
    for (key, m, k), want in cases.items():
        assert O.py_indexes(key, m, k) == want
        assert oracle.indexes(key, m, k) == want


def test_golden_indexes(golden, O, oracle):
    for v in golden["indexes"]:
        kb = bytes.fromhex(v["key_hex"])
        assert O.py_indexes(kb, v["m"], v["k"]) == v["idx"]
        assert oracle.indexes(kb, v["m"], v["k"]) == v["idx"]


def test_golden_strings(golden, O, oracle):
    for s in golden["strings"]:
        m, k = s["m"], s["k"]
        ib, io = O.pack_keys(s["insert"])
        bits = oracle.new_bitset(m, k)
        any_new, per_key = oracle.insert_many(bits, m, k, ib, io, per_key=True)
        rs = oracle.redis_string(bits)
        assert len(rs) == s["redis_len"]
        assert hashlib.sha1(rs).hexdigest() == s["redis_sha1"]
        if s["redis_hex"] is not None:
            assert rs.hex() == s["redis_hex"]
        assert per_key.tolist() == s["sequential_new"]
        assert any_new == any(s["sequential_new"])
        pb, po = O.pack_keys(s["probe"])
        assert oracle.include_many(bits, m, k, pb, po).tolist() == s["include"]


def test_survey_strings(O, oracle):
    bits = oracle.new_bitset(9585, 6)
    ib, io = O.pack_keys(["asdlol"])
    oracle.insert_many(bits, 9585, 6, ib, io)
    s = oracle.redis_string(bits)
    assert (len(s), hashlib.sha1(s).hexdigest()) == (1101, "fdb117fe21dea15cb79ef9decc983623b10f8af9")


def test_ruby_driver_restatement_matches_c(O, oracle, pkg):
    """RubyDriverRestatement over FakeRedis (SETBIT path) == C oracle bitset."""
    r = pkg.FakeRedis()
    opts = {"bits": 95851, "hashes": 6, "key_name": "bf", "redis": r}
    drv = O.RubyDriverRestatement(opts)
    keys = ["k%d" % i for i in range(700)]
    for key in keys:
        drv.insert(key)
    bits = oracle.new_bitset(95851, 6)
    ib, io = O.pack_keys(keys)
    oracle.insert_many(bits, 95851, 6, ib, io)
    assert r.get("bf") == oracle.redis_string(bits)
    assert all(drv.include(k) for k in keys)


def test_omp_matches_sequential(O, oracle):
    rng = np.random.default_rng(3)
    vals = rng.integers(0, 10**7, 200_000)
    ib, io = O.pack_keys([int(v) for v in vals[:20000]])
    for m, k in ((95851, 6), (9585058, 6)):
        a = oracle.new_bitset(m, k)
        b = oracle.new_bitset(m, k)
        oracle.insert_many(a, m, k, ib, io)
        oracle.insert_many_omp(b, m, k, ib, io, 4)
        assert np.array_equal(a, b)
        np.testing.assert_array_equal(oracle.include_many(a, m, k, ib, io),
                                      oracle.include_many_omp(a, m, k, ib, io, 4))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_node_crosscheck():
    out = subprocess.run(["node", os.path.join(HERE, "golden", "crosscheck_node.js")],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


def test_golden_file_is_current():
    out = subprocess.run(["python", os.path.join(HERE, "golden", "make_golden.py"), "--check"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr


def test_rfc1321_md5(golden, O):
    """The RubyTest engines' MD5 (ruby_test.rb:55-57) is RFC 1321's: its appendix A.5 suite."""
    assert golden["rfc1321_md5"] == O.RFC1321_MD5
    for msg, want in O.RFC1321_MD5.items():
        assert hashlib.md5(msg.encode()).hexdigest() == want


def test_golden_engine_indexes(golden, O):
    """ruby_test.rb:43-61 restated (py_engine_indexes) against the committed vectors."""
    assert len(golden["engine_indexes"]) == 448
    for v in golden["engine_indexes"]:
        got = O.py_engine_indexes(bytes.fromhex(v["key_hex"]), int(v["m"]), v["k"], v["engine"])
        assert got == [int(x) for x in v["idx"]]
    # hand-checkable anchor: probe 0 of "asdlol" = int(md5("0-asdlol")) mod m
    assert O.py_engine_indexes("asdlol", 9585, 1, "md5") == [int(hashlib.md5(b"0-asdlol").hexdigest(), 16) % 9585]
    with pytest.raises(O.ArgumentError_):
        O.py_engine_indexes("x", 100, 3, "crc32")

"""spec/redis_bloomfilter_spec.rb:89-120, which runs its four cases for every driver
(`%w[ruby lua ruby-test]`), run for the three device drivers that stand in for them:
'hip' (ruby.rb), 'hip-lua' (lua.rb + add.lua / check.lua) and 'hip-test' (ruby_test.rb),
over FakeRedis standing in for Redis.current."""
import random

import pytest

pytestmark = pytest.mark.gpu

DRIVERS = ["hip", "hip-lua", "hip-test"]


def factory(pkg, options, driver, redis):   # spec:19-22
    options = dict(options, driver=driver, redis=redis)
    return pkg.Bloomfilter(options)


def error_rate(bf, elems, rng):   # spec:7-17
    visited = set()
    error = 0
    for _ in range(elems):
        a = rng.randrange(elems)
        if bf.include(a) != (a in visited):
            error += 1
        visited.add(a)
        bf.insert(a)
    return error / elems


@pytest.mark.parametrize("driver", DRIVERS)
def test_should_work(pkg, driver):   # spec:90-98
    bf = factory(pkg, {"size": 1000, "error_rate": 0.01, "key_name": "__test_bf"}, driver, pkg.FakeRedis())
    bf.clear()
    assert bf.include("asdlol") is False
    bf.insert("asdlol")
    assert bf.include("asdlol") is True
    bf.clear()
    assert bf.include("asdlol") is False


@pytest.mark.parametrize("driver", DRIVERS)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_should_honor_the_error_rate(pkg, driver, seed):   # spec:100-106
    bf = factory(pkg, {"size": 100, "error_rate": 0.02, "key_name": "__test_bf"}, driver, pkg.FakeRedis())
    bf.clear()
    e = error_rate(bf, 180, random.Random(seed))
    assert round(e, 2) <= round(bf.options["error_rate"], 2)
    bf.clear()


@pytest.mark.parametrize("driver", DRIVERS)
def test_should_add_an_element(pkg, driver):   # spec:108-112
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "__test_bf"}, driver, pkg.FakeRedis())
    bf.insert("asdlolol")
    assert bf.include("asdlolol") is True


@pytest.mark.parametrize("driver", DRIVERS)
def test_should_add_ttl_when_requested(pkg, driver):   # spec:114-118 (the lua layout's key is name:1)
    r = pkg.FakeRedis()
    bf = factory(pkg, {"size": 100, "error_rate": 0.01, "key_name": "__test_bf_%s" % driver}, driver, r)
    bf.insert("asdlolol", 120)
    assert r.ttl("__test_bf_%s%s" % (driver, ":1" if driver == "hip-lua" else "")) > 0


@pytest.mark.parametrize("driver", DRIVERS)
def test_insert_with_expire_zero(pkg, driver):
    """insert(x, 0): 0 is truthy in Ruby (bloomfilter.rb:62, ruby.rb:62) and in Lua
    (tonumber(ARGV[4]), add.lua:4, 51), so the reference EXPIREs the key with 0 and Redis
    deletes it; include? then reads a missing key -> false.  A later insert without expire
    rebuilds the key with no TTL.  Checked against the restatements on their own FakeRedis."""
    import lua_oracle
    import oracle as O
    r, r_ref = pkg.FakeRedis(), pkg.FakeRedis()
    name = "__test_bf_exp0_%s" % driver
    bf = factory(pkg, {"size": 1000, "error_rate": 0.01, "key_name": name}, driver, r)
    key = name + (":1" if driver == "hip-lua" else "")
    bf.insert("asdlolol", 0)
    assert r.exists(key) == 0
    assert bf.include("asdlolol") is False
    if driver == "hip":
        ref = O.RubyDriverRestatement({"bits": bf.options["bits"], "hashes": bf.options["hashes"],
                                       "key_name": name, "redis": r_ref})
        ref.insert("asdlolol", 0)
        assert ref.include("asdlolol") is False and r_ref.exists(name) == 0
    elif driver == "hip-lua":
        lua_oracle.add(r_ref, name, 1000, 0.01, "asdlolol", 0)
        assert lua_oracle.check(r_ref, name, 1000, 0.01, "asdlolol") is False
        assert r.get(name + ":count") == r_ref.get(name + ":count") == b"1"   # the count has no TTL
    bf.insert("asdlolol")
    assert bf.include("asdlolol") is True
    assert r.exists(key) == 1 and r.ttl(key) == -1
    if driver == "hip":
        ref.insert("asdlolol")
        assert r.get(name) == r_ref.get(name)

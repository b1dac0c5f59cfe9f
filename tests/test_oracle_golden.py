"""Pins the CPU oracle against the reference's own known answers (CPU only).

tests/golden/reference_vectors.json holds vectors transcribed from the reference's
test/redis/fixed_cache_impl_test.go, test/limiter/base_limiter_test.go and
test/integration/integration_test.go (see tests/golden/make_golden.py).
"""
import numpy as np
import pytest

import hiprl
import oracle
import streams


def test_decide_vectors(golden):
    ratio = golden["near_limit_ratio"]
    for v in golden["decide"]:
        st, thr = oracle.decide(v["L"], v["unit"], ratio, v["now"], v["hits"], v["after"], v["local_hit"],
                                v["has_limit"], v["before"])
        e = v["expect"]
        cf = int(st["code_flags"])
        got = dict(code=cf & 0xFF, remaining=int(st["limit_remaining"]), reset=int(st["reset_s"]),
                   over=int(st["over_limit_delta"]), near=int(st["near_limit_delta"]), throttle=thr)
        assert got == e, v["src"]
        assert bool((cf >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT) == v["local_hit"], v["src"]


def test_cache_keys(golden):
    for v in golden["keys"]:
        prefix = hiprl.cache_key_prefix(v["domain"], v["entries"])
        assert oracle.cache_key(prefix, v["unit"], v["now"]).decode() == v["key"], v["src"]


@pytest.mark.parametrize("split", ["one_batch", "per_request", "uneven"])
def test_integration_streams(golden, split):
    for s in golden["streams"]:
        n = len(s["requests"])
        sizes = {"one_batch": None, "per_request": [1] * n, "uneven": [3, 1, 7, 2, n - 13]}[split]
        streams.check_integration_stream(oracle.Oracle(local_cache=s["local_cache"]), s, sizes)


def test_local_cache_check_stream(golden):
    for s in golden["check_streams"]:
        streams.check_check_stream(oracle.Oracle(local_cache=s["local_cache"]), s)
        streams.check_check_stream(oracle.Oracle(local_cache=s["local_cache"]), s, [1] * len(s["requests"]))


def test_decide_vectors_as_streams(golden):
    """The DoLimit-path decide vectors replayed as request streams on the stream oracle."""
    ratio = golden["near_limit_ratio"]
    n = 0
    for v in golden["decide"]:
        x = streams.decide_as_stream(v)
        if x is None:
            continue
        rules, reqs, k = x
        o = oracle.Oracle(near_limit_ratio=ratio, local_cache=v["local_hit"])
        o.load_rules(rules)
        st, thr = streams.replay(o, reqs)
        e = v["expect"]
        s = st[k]
        got = dict(code=int(s["code_flags"]) & 0xFF, remaining=int(s["limit_remaining"]), reset=int(s["reset_s"]),
                   over=int(s["over_limit_delta"]), near=int(s["near_limit_delta"]), throttle=int(thr[k]))
        assert got == e, v["src"]
        n += 1
    assert n >= 14


def test_duplicate_descriptors_in_one_request():
    """Both descriptors INCRBY (fixed_cache_impl.go:55-86 checks the local cache for all
    descriptors before any Set): 2 hits on L=1 give post-values 1 and 2."""
    o = oracle.Oracle(local_cache=True)
    o.load_rules([(1, hiprl.SECOND)])
    ent = [("k", "v")]
    st, _ = streams.replay(o, [("d", [ent, ent], [0, 0], 1, 100), ("d", [ent], [0], 1, 100)])
    codes = [int(x) & 0xFF for x in st["code_flags"]]
    assert codes == [hiprl.CODE_OK, hiprl.CODE_OVER_LIMIT, hiprl.CODE_OVER_LIMIT]
    assert (int(st["code_flags"][2]) >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT
    assert o.counter(b"d_k_v_100") == 2


def test_key_string_collision_shares_counter():
    """("a_b","c") and ("a","b_c") produce the same key string (cache_key.go:57-65)."""
    o = oracle.Oracle()
    o.load_rules([(10, hiprl.MINUTE)])
    st, _ = streams.replay(o, [("d", [[("a_b", "c")]], [0], 1, 120), ("d", [[("a", "b_c")]], [0], 1, 130)])
    assert [int(x) for x in st["limit_remaining"]] == [9, 8]


def test_multithreaded_oracle_matches_serial():
    rng = np.random.default_rng(7)
    reqs = []
    for r in range(3000):
        nd = int(rng.integers(1, 4))
        descs = [[("k", str(int(rng.integers(0, 50))))] for _ in range(nd)]
        rules = [int(rng.integers(0, 3)) if rng.random() > 0.1 else streams.NIL for _ in range(nd)]
        reqs.append(("dom", descs, rules, int(rng.integers(0, 4)), 1000 + r // 500))
    b = hiprl.build_batch(reqs)
    outs = []
    for th in (1, 4):
        o = oracle.Oracle(local_cache=True)
        o.load_rules([(5, hiprl.SECOND), (30, hiprl.MINUTE), (100, hiprl.HOUR)])
        outs.append(o.submit(b, threads=th))
    streams.assert_same(*outs[0], *outs[1], "mt vs serial")

"""Shared helpers: replay golden streams and synthetic streams through a backend.

A backend is any object with load_rules(rules) and submit(batch) -> (status, throttle),
i.e. oracle.Oracle (CPU restatement) or hiprl.Engine (HIP path via the C ABI).
"""
from __future__ import annotations

import zlib

import numpy as np

import hiprl

NIL = hiprl.NIL_RULE


def fixture_requests(stream):
    out = []
    for r in stream["requests"]:
        rules = [NIL if x is None else x for x in r["rules"]]
        descs = [[tuple(e) for e in d] for d in r["descriptors"]]
        out.append((r["domain"], descs, rules, r["hits"], r["now"]))
    return out


def replay(backend, reqs, batch_sizes=None):
    """Submit `reqs` in consecutive batches (default: all in one batch). Returns the
    concatenated per-descriptor status array and per-request throttle array."""
    if batch_sizes is None:
        batch_sizes = [len(reqs)]
    sts, thrs = [], []
    i = 0
    for bs in batch_sizes:
        if bs == 0:
            continue
        st, thr = backend.submit(hiprl.build_batch(reqs[i:i + bs]))
        sts.append(st)
        thrs.append(thr)
        i += bs
    assert i == len(reqs)
    return np.concatenate(sts), np.concatenate(thrs)


def check_integration_stream(backend, stream, batch_sizes=None):
    """Assert the per-request statuses and cumulative stats of an integration stream."""
    reqs = fixture_requests(stream)
    backend.load_rules([tuple(x) for x in stream["rules"]])
    st, thr = replay(backend, reqs, batch_sizes)
    stats = {}
    d = 0
    for r, (req, exp) in enumerate(zip(stream["requests"], stream["expect"])):
        for k, (rule, (code, remaining, has_limit)) in enumerate(zip(req["rules"], exp["statuses"])):
            s = st[d]
            d += 1
            cf = int(s["code_flags"])
            assert cf & 0xFF == code, (exp["src"], k, cf)
            assert int(s["limit_remaining"]) == remaining, (exp["src"], k, int(s["limit_remaining"]))
            assert bool((cf >> 8) & hiprl.FLAG_HAS_LIMIT) == has_limit, (exp["src"], k)
            if rule is None:
                continue
            name = stream["stat_keys"][rule]
            c = stats.setdefault(name, dict(total_hits=0, over_limit=0, near_limit=0,
                                            over_limit_with_local_cache=0))
            c["total_hits"] += max(1, req["hits"])
            c["over_limit"] += int(s["over_limit_delta"])
            c["near_limit"] += int(s["near_limit_delta"])
            if (cf >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT:
                c["over_limit_with_local_cache"] += int(s["over_limit_delta"])
        for name, want in exp["stats"].items():
            for k, v in want.items():
                assert stats[name][k] == v, (exp["src"], name, k, stats[name][k], v)
    return st, thr


def check_check_stream(backend, stream, batch_sizes=None):
    reqs = fixture_requests(stream)
    backend.load_rules([tuple(x) for x in stream["rules"]])
    st, thr = replay(backend, reqs, batch_sizes)
    for r, chk in enumerate(stream["checks"]):
        if chk is None:
            continue
        s = st[r]  # one descriptor per request
        cf = int(s["code_flags"])
        assert [cf & 0xFF, int(s["limit_remaining"])] == chk["status"], chk["src"]
        local = bool((cf >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT)
        got = dict(over=int(s["over_limit_delta"]), near=int(s["near_limit_delta"]),
                   olwlc=int(s["over_limit_delta"]) if local else 0)
        assert got == chk["delta"], (chk["src"], got)
        assert int(thr[r]) == chk["throttle"], (chk["src"], int(thr[r]))


def decide_as_stream(v):
    """A decide vector on the DoLimit path (before = after - hits) as a request stream on a
    fresh key: a warm-up request brings the counter to after - hits, then the checked one.
    A local-cache-hit vector is reached by a warm-up that goes over the limit first.
    Returns (rules, requests, index of the checked request) or None if unreachable."""
    if v["before"] is not None or not v["has_limit"]:
        return None
    dom, ent = "golden", [("key", f"v{v['L']}_{v['unit']}_{v['after']}_{v['hits']}_{int(v['local_hit'])}")]
    reqs = []
    if v["local_hit"]:
        reqs.append((dom, [ent], [0], v["L"] + 1, v["now"]))
    else:
        pre = v["after"] - v["hits"]
        if pre < 0:
            return None
        if pre > 0:
            reqs.append((dom, [ent], [0], pre, v["now"]))
    reqs.append((dom, [ent], [0], v["hits"], v["now"]))
    return [(v["L"], v["unit"])], reqs, len(reqs) - 1


def assert_same(a_st, a_thr, b_st, b_thr, ctx=""):
    """Bit-exact comparison of two (status, throttle) outputs, with a readable first diff."""
    if not np.array_equal(a_st, b_st):
        bad = np.nonzero(a_st != b_st)[0]
        i = int(bad[0])
        raise AssertionError(f"{ctx}: {len(bad)} descriptor statuses differ; first at {i}: {a_st[i]} vs {b_st[i]}")
    if not np.array_equal(a_thr, b_thr):
        bad = np.nonzero(a_thr != b_thr)[0]
        i = int(bad[0])
        raise AssertionError(f"{ctx}: {len(bad)} request throttles differ; first at {i}: {a_thr[i]} vs {b_thr[i]}")


# ---------------------------------------------------------------------------
# Seeded random request streams (parity tests, router tests)
# ---------------------------------------------------------------------------
UNITS = [hiprl.SECOND, hiprl.MINUTE, hiprl.HOUR, hiprl.DAY]
LS = [1, 3, 10, 40]  # limits per unit -> rule id = u * len(LS) + l
RULES = [(L, u) for u in UNITS for L in LS]


def make_stream(seed, n_req, t0, keyspace=40, max_desc=4, nil_p=0.08, override_p=0.05, dt_max=2):
    rng = np.random.default_rng(seed)
    reqs = []
    t = t0
    for _ in range(n_req):
        if rng.random() < 0.02:
            t += int(rng.integers(1, dt_max + 1))
        dom = ["dom", "a", "a_b"][int(rng.integers(0, 3))]
        nd = int(rng.integers(1, max_desc + 1))
        descs, rules = [], []
        for _ in range(nd):
            kind = rng.random()
            if kind < 0.1:  # colliding entry splits: same key string
                descs.append([("a_b", "c")] if rng.random() < 0.5 else [("a", "b_c")])
            else:
                ne = int(rng.integers(1, 4))
                descs.append([(f"k{j}", f"v{int(rng.integers(0, keyspace))}") for j in range(ne)])
            if rng.random() < nil_p:
                rules.append(NIL)
                continue
            prefix = hiprl.cache_key_prefix(dom, descs[-1])
            hsh = zlib.crc32(prefix)
            u = hsh % 4  # the unit is a function of the key string
            li = (hsh >> 8) % len(LS)
            if rng.random() < override_p:
                li = int(rng.integers(0, len(LS)))
            rules.append(u * len(LS) + li)
        if rng.random() < 0.05 and nd > 0:  # duplicate a descriptor inside the request
            descs.append(descs[0])
            rules.append(rules[0])
        reqs.append((dom, descs, rules, int(rng.integers(0, 9)), t))
    return reqs


def batch_sizes(reqs, rng, max_bs):
    """Random batch cuts that keep each batch within two adjacent seconds."""
    sizes, i = [], 0
    while i < len(reqs):
        bs = int(rng.integers(1, max_bs + 1))
        j = i + 1
        t_lo = reqs[i][4]
        while j < len(reqs) and j - i < bs and reqs[j][4] - t_lo <= 1:
            j += 1
        sizes.append(j - i)
        i = j
    return sizes

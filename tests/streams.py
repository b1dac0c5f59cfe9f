"""Shared helpers: replay golden streams and synthetic streams through a backend.

A backend is any object with load_rules(rules) and submit(batch) -> (status, throttle),
i.e. oracle.Oracle (CPU restatement) or hiprl.Engine (HIP path via the C ABI).
"""
from __future__ import annotations

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

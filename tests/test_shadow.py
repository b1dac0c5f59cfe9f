"""Shadow mode (BASELINE config 4) — an extension: this fork has no shadow mode (its YAML
validator rejects a `shadow_mode` key, src/config/config_impl.go:49-59), so there is no
reference fixture and parity is unpinned. Definition (following
envoyproxy/ratelimit's later GetResponseDescriptorStatus): a rule flagged RL_RULE_SHADOW never
answers OVER_LIMIT; such a decision is answered OK with RL_FLAG_SHADOW (Stats.ShadowMode + 1)
while counters, the local-cache freeze, LimitRemaining, reset and the over/near stat deltas
stay those of the OVER_LIMIT decision.

CPU: the oracle's known answers and the property that a shadow stream equals the plain stream
with every OVER_LIMIT code rewritten. GPU: the HIP path bit-exact against the oracle on mixed
shadow / enforced rules (v4 and LSD pipelines, hot keys, local cache on and off) and through
the Python DoLimit mirror's stats.
"""
import numpy as np
import pytest

import hiprl
import oracle
import streams
from streams import RULES, batch_sizes, make_stream

T0 = 1_700_000_000
OK, OVER = hiprl.CODE_OK, hiprl.CODE_OVER_LIMIT
SHADOW = hiprl.FLAG_SHADOW << 8
RULES_SHADOW = [(L, u, k % 2 == 1) for k, (L, u) in enumerate(RULES)]


def shadowed(st, rules, reqs):
    """The plain decisions with shadow applied: every OVER_LIMIT of a shadow rule -> OK | SHADOW."""
    rule_ids = np.array([r for _, descs, rl, _, _ in reqs for r in rl], np.int64)
    out = st.copy()
    cf = out["code_flags"]
    sh = np.array([bool(rules[r][2]) if r != streams.NIL else False for r in rule_ids])
    m = sh & ((cf & 0xFF) == OVER)
    out["code_flags"] = np.where(m, (cf & ~np.uint32(0xFF)) | OK | SHADOW, cf)
    return out


def _oracle(rules, local_cache):
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(rules)
    return o


@pytest.mark.parametrize("local_cache", [False, True])
def test_oracle_known_answers(local_cache):
    """L = 2 per SECOND, shadow: hits 1, 2 OK; hit 3 over -> OK|SHADOW with over_limit_delta 1;
    with the local cache on, hit 4 is a local-cache hit (no INCRBY) -> OK|SHADOW|LOCAL_CACHE_HIT;
    the enforced twin rule answers OVER_LIMIT at the same points."""
    rules = [(2, hiprl.SECOND, True), (2, hiprl.SECOND, False)]
    for rule, want_over in ((0, OK), (1, OVER)):
        o = _oracle(rules, local_cache)
        reqs = [("d", [[("k", "v")]], [rule], 1, T0)] * 4
        st, thr = streams.replay(o, reqs, [1, 1, 1, 1])
        codes = [int(c) & 0xFF for c in st["code_flags"]]
        flags = [int(c) >> 8 for c in st["code_flags"]]
        assert codes == [OK, OK, want_over, want_over]
        assert list(st["limit_remaining"]) == [1, 0, 0, 0]
        assert list(st["over_limit_delta"]) == [0, 0, 1, 1]
        assert list(st["near_limit_delta"]) == [0, 1, 0, 0]
        sh = hiprl.FLAG_SHADOW if rule == 0 else 0
        lc = hiprl.FLAG_LOCAL_CACHE_HIT if local_cache else 0
        assert flags == [1, 1, 1 | sh, 1 | sh | lc]
        # the counter advanced on every hit except the local-cache one
        assert o.counter(b"d_k_v_%d" % T0, T0) == (3 if local_cache else 4)


@pytest.mark.parametrize("local_cache", [False, True])
def test_oracle_shadow_is_a_code_rewrite(local_cache):
    """Same stream, shadow vs plain rules: identical except OVER_LIMIT codes of shadow rules."""
    reqs = make_stream(7, 5000, t0=T0 - 40)
    sizes = batch_sizes(reqs, np.random.default_rng(70), 1200)
    plain = streams.replay(_oracle(RULES, local_cache), reqs, sizes)
    shadow = streams.replay(_oracle(RULES_SHADOW, local_cache), reqs, sizes)
    want = shadowed(plain[0], RULES_SHADOW, reqs)
    assert np.array_equal(shadow[0], want)
    assert np.array_equal(shadow[1], plain[1])
    assert int(((shadow[0]["code_flags"] >> 8) & hiprl.FLAG_SHADOW).astype(bool).sum()) > 0


def test_shadow_bit_validation():
    o = oracle.Oracle()
    with pytest.raises(ValueError):
        o.load_rules([(5, 0, True)])  # shadow on an invalid unit is still invalid


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["v4", "lsd"])
@pytest.mark.parametrize("local_cache", [False, True])
def test_gpu_shadow_streams(local_cache, pipeline):
    reqs = make_stream(21, 6000, t0=T0 - 90)
    sizes = batch_sizes(reqs, np.random.default_rng(22), 1500)
    o = _oracle(RULES_SHADOW, local_cache)
    e = hiprl.Engine(local_cache=local_cache, max_batch_desc=1 << 17, pipeline=pipeline)
    e.load_rules(RULES_SHADOW)
    ost, othr = streams.replay(o, reqs, sizes)
    gst, gthr = streams.replay(e, reqs, sizes)
    streams.assert_same(ost, othr, gst, gthr, f"shadow local={local_cache} pipeline={pipeline}")
    assert int(((gst["code_flags"] >> 8) & hiprl.FLAG_SHADOW).astype(bool).sum()) > 0
    assert int(((gst["code_flags"] & 0xFF) == OVER).sum()) > 0  # enforced rules still answer OVER_LIMIT


@pytest.mark.gpu
@pytest.mark.parametrize("local_cache", [False, True])
def test_gpu_shadow_hot_keys(local_cache):
    """Hot keys (decided in place by k4_place, deferred ones by k4_group) under shadow rules."""
    from test_gpu_parity import hot_stream

    reqs, sizes = hot_stream(5, 12000, t0=T0 - 2, seed=5 + local_cache)
    o = _oracle(RULES_SHADOW, local_cache)
    e = hiprl.Engine(local_cache=local_cache, max_batch_desc=1 << 17)
    e.load_rules(RULES_SHADOW)
    ost, othr = streams.replay(o, reqs, sizes)
    gst, gthr = streams.replay(e, reqs, sizes)
    streams.assert_same(ost, othr, gst, gthr, f"shadow hot local={local_cache}")
    assert e.stats()["hot_keys"] >= 2
    assert int(((gst["code_flags"] >> 8) & hiprl.FLAG_SHADOW).astype(bool).sum()) > 1000


@pytest.mark.gpu
def test_gpu_mirror_shadow_stats():
    """HipRateLimitCache (the DoLimit mirror): a shadow limit answers OK and counts ShadowMode."""
    now = [T0]
    cache = hiprl.HipRateLimitCache(lambda: now[0], local_cache=True)
    scope = hiprl.StatsStore()
    sh = hiprl.NewRateLimit(3, hiprl.SECOND, "key_shadow", scope, shadow_mode=True)
    en = hiprl.NewRateLimit(3, hiprl.SECOND, "key_enforced", scope)
    req = hiprl.NewRateLimitRequest("domain", [[("a", "b")], [("c", "d")]], 1)
    codes = []
    for _ in range(6):
        r = cache.DoLimit(req, [sh, en])
        codes.append([s.Code for s in r.DescriptorStatuses])
    assert codes == [[OK, OK]] * 3 + [[OK, OVER]] * 3
    assert sh.Stats.ShadowMode.Value() == 3 and en.Stats.ShadowMode.Value() == 0
    assert sh.Stats.OverLimit.Value() == en.Stats.OverLimit.Value() == 3
    assert sh.Stats.OverLimitWithLocalCache.Value() == en.Stats.OverLimitWithLocalCache.Value() == 2
    assert sh.Stats.NearLimit.Value() == en.Stats.NearLimit.Value()


@pytest.mark.gpu
def test_gpu_mirror_shadow_stats_hits_addend():
    """Stats.ShadowMode with hits_addend 4. It counts shadowed DECISIONS (+1
    each, as upstream envoyproxy/ratelimit's GetResponseDescriptorStatus does with
    `limitInfo.limit.Stats.ShadowMode.Inc()` — upstream is not in /root/reference, so this is
    parity unpinned), while the over / near / local-cache stats grow by hits as for an enforced
    rule. L = 10/SECOND, ratio 0.8 (near 8): posts 4, 8 OK; post 12 over (checkOverLimitThreshold,
    base_limiter.go:129-145: OverLimit += 12 - 10, NearLimit += 10 - max(8, 8)), then a
    local-cache hit (OverLimit += 4, OverLimitWithLocalCache += 4): ShadowMode 2."""
    now = [T0]
    cache = hiprl.HipRateLimitCache(lambda: now[0], local_cache=True)
    scope = hiprl.StatsStore()
    sh = hiprl.NewRateLimit(10, hiprl.SECOND, "key_shadow4", scope, shadow_mode=True)
    en = hiprl.NewRateLimit(10, hiprl.SECOND, "key_enforced4", scope)
    req = hiprl.NewRateLimitRequest("domain", [[("a", "b")], [("c", "d")]], 4)
    codes = []
    for _ in range(4):
        r = cache.DoLimit(req, [sh, en])
        codes.append([s.Code for s in r.DescriptorStatuses])
    assert codes == [[OK, OK]] * 2 + [[OK, OVER]] * 2
    assert sh.Stats.ShadowMode.Value() == 2 and en.Stats.ShadowMode.Value() == 0
    assert sh.Stats.OverLimit.Value() == en.Stats.OverLimit.Value() == 2 + 4
    assert sh.Stats.OverLimitWithLocalCache.Value() == en.Stats.OverLimitWithLocalCache.Value() == 4
    assert sh.Stats.NearLimit.Value() == en.Stats.NearLimit.Value()
    assert sh.Stats.TotalHits.Value() == en.Stats.TotalHits.Value() == 16

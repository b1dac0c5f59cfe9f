"""The reference's known answers replayed through the HIP path (C ABI on an MI355X)."""
import numpy as np
import pytest

import hiprl
import streams

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("split", ["one_batch", "per_request", "uneven"])
def test_integration_streams_gpu(golden, split):
    for s in golden["streams"]:
        n = len(s["requests"])
        sizes = {"one_batch": None, "per_request": [1] * n, "uneven": [3, 1, 7, 2, n - 13]}[split]
        streams.check_integration_stream(hiprl.Engine(local_cache=s["local_cache"]), s, sizes)


def test_local_cache_check_stream_gpu(golden):
    for s in golden["check_streams"]:
        streams.check_check_stream(hiprl.Engine(local_cache=True), s)
        streams.check_check_stream(hiprl.Engine(local_cache=True), s, [1] * len(s["requests"]))


@pytest.mark.parametrize("one_batch", [True, False])
def test_decide_vectors_gpu(golden, one_batch):
    ratio = golden["near_limit_ratio"]
    n = 0
    for v in golden["decide"]:
        x = streams.decide_as_stream(v)
        if x is None:
            continue
        rules, reqs, k = x
        eng = hiprl.Engine(near_limit_ratio=ratio, local_cache=v["local_hit"])
        eng.load_rules(rules)
        st, thr = streams.replay(eng, reqs, None if one_batch else [1] * len(reqs))
        e = v["expect"]
        s = st[k]
        got = dict(code=int(s["code_flags"]) & 0xFF, remaining=int(s["limit_remaining"]), reset=int(s["reset_s"]),
                   over=int(s["over_limit_delta"]), near=int(s["near_limit_delta"]), throttle=int(thr[k]))
        assert got == e, v["src"]
        n += 1
    assert n >= 14


def test_reference_style_cache_mirror():
    """TestNearLimit-style scenario through the DoLimit mirror (fixed_cache_impl_test.go:275-339)."""
    store = hiprl.StatsStore()
    cache = hiprl.HipRateLimitCache(lambda: 1000000)
    limits = [hiprl.NewRateLimit(15, hiprl.HOUR, "key4_value4", store)]
    req = hiprl.NewRateLimitRequest("domain", [[("key4", "value4")]], 1)
    resps = [cache.DoLimit(req, limits) for _ in range(16)]
    r11, r13, r16 = resps[10], resps[12], resps[15]
    assert r11.DescriptorStatuses[0] == hiprl.DescriptorStatus(hiprl.CODE_OK, limits[0].Limit, 4, 800)
    assert r13.DescriptorStatuses[0] == hiprl.DescriptorStatus(hiprl.CODE_OK, limits[0].Limit, 2, 800)
    assert r13.ThrottleMillis == 400000
    assert r16.DescriptorStatuses[0] == hiprl.DescriptorStatus(hiprl.CODE_OVER_LIMIT, limits[0].Limit, 0, 800)
    assert limits[0].Stats.TotalHits.Value() == 16
    assert limits[0].Stats.OverLimit.Value() == 1
    assert limits[0].Stats.NearLimit.Value() == 3  # posts 13, 14, 15


def test_nil_limit_and_empty_batch():
    eng = hiprl.Engine()
    eng.load_rules([(10, hiprl.SECOND)])
    st, thr = eng.submit(hiprl.build_batch([("d", [[("a", "b")], [("c", "d")]], [streams.NIL, 0], 1, 5)]))
    assert int(st["code_flags"][0]) == hiprl.CODE_OK and int(st["limit_remaining"][0]) == 0
    assert int(st["reset_s"][0]) == 0
    assert int(st["code_flags"][1]) & 0xFF == hiprl.CODE_OK and int(st["limit_remaining"][1]) == 9
    st, thr = eng.submit(hiprl.build_batch([]))
    assert st.shape == (0,) and thr.shape == (0,)

"""REDIS_PERSECOND: SECOND keys in their own store.

With `perSecondClient` set, a SECOND key and a MINUTE key with the same string are
different counters (`src/redis/fixed_cache_impl.go:74-85`). The HIP table always keeps every
unit in its own key space, so it reproduces the split configuration exactly:
the GPU test drives same-string SECOND and MINUTE keys (window starts that coincide at a
minute boundary) and checks bit-exactness against the oracle with the split on. Without the split,
Redis shares such a counter and its TTL follows whichever EXPIRE came last (wall clock); the
CPU test shows the oracle's shared-counter behaviour, which the device does not claim. The
local over-limit cache is one freecache keyed by the key string for both clients
(`src/limiter/base_limiter.go:57-66,94-106`), so with it on a SECOND key that goes over limit
also freezes the MINUTE key of the same string; the device freezes per unit, so that case is
outside the claim too (measured: 57 of the local-cache stream's statuses differ)."""
import numpy as np
import pytest

import hiprl
import oracle
from streams import assert_same, batch_sizes, replay

T0 = 1_699_999_200  # a multiple of 3600: SECOND, MINUTE and HOUR windows all start here
RULES = [(5, hiprl.SECOND), (40, hiprl.MINUTE), (90, hiprl.HOUR)]


def same_string_stream(seed, n_req=240):
    rng = np.random.default_rng(seed)
    reqs, t = [], T0
    for q in range(n_req):
        if q and q % 60 == 0:
            t += 1  # the SECOND window moves on; MINUTE/HOUR keep the T0 string
        descs, rules = [], []
        for _ in range(int(rng.integers(1, 4))):
            r = int(rng.integers(0, 3))
            # SECOND and MINUTE share key strings; HOUR keys use their own (a MINUTE and an
            # HOUR key with one string share a counter even with the split: not claimed)
            descs.append([("k" if r < 2 else "h", f"v{int(rng.integers(0, 3))}")])
            rules.append(r)
        reqs.append(("dom", descs, rules, int(rng.integers(0, 4)), t))
    return reqs


def test_same_string_keys_split_vs_shared_oracle():
    reqs = same_string_stream(1)
    split, shared = oracle.Oracle(per_second_split=True), oracle.Oracle(per_second_split=False)
    split.load_rules(RULES)
    shared.load_rules(RULES)
    a = replay(split, reqs)
    b = replay(shared, reqs)
    key = b"dom_k_v0_%d" % T0
    # the split keeps the SECOND counter apart; the shared store sums every unit's hits
    assert shared.counter(key) == split.counter(key) + split.counter(key, per_second=True)
    assert not np.array_equal(a[0], b[0])


@pytest.mark.gpu
@pytest.mark.parametrize("local_cache", [False])
def test_gpu_matches_split_oracle_on_same_string_keys(local_cache):
    reqs = same_string_stream(2 + local_cache)
    sizes = batch_sizes(reqs, np.random.default_rng(7), 50)
    o = oracle.Oracle(local_cache=local_cache, per_second_split=True)
    o.load_rules(RULES)
    e = hiprl.Engine(local_cache=local_cache, per_second_split=True)
    e.load_rules(RULES)
    assert_same(*replay(e, reqs, sizes), *replay(o, reqs, sizes), ctx=f"per-second split lc={local_cache}")

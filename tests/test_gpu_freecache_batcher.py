"""HIP_LOCAL_CACHE=freecache: the single-engine batcher (HipRateLimitCache) with its local
over-limit cache held in the host's bounded freecache model (rl_freecache.hpp) instead of the
device's cache, against a serial DoLimit of the reference (fixed_cache_impl.go:31-123 +
base_limiter.go:57-195) whose local cache is the Python restatement of freecache
(tests/freecache_model.py).

The serial model is first pinned against the device's own local cache (the product default,
bit-exact against the oracle in test_gpu_cache_mirror.py): with a cache large enough never to
evict, freecache and the device cache must give the same statuses and stats. Then a 512-KiB
cache (freecache's floor) holds a fraction of the over-limit keys, so entries are evicted and
evicted keys INCRBY again; statuses, per-rule stats and the cache's counters must equal the
model's. The eviction itself is PARITY UNPINNED (freecache is not in this image)."""
import ctypes as C
import math

import numpy as np
import pytest

import hiprl
from freecache_model import FreeCache
from test_gpu_cache_mirror import Mirror, _lib

pytestmark = pytest.mark.gpu


class FcMirror(Mirror):
    def __init__(self, size, ratio=0.8):
        self.lib = _lib()
        self.lib.rlc_create_fc.argtypes = [C.c_int64, C.c_float, C.c_int, C.c_uint32]
        self.lib.rlc_create_fc.restype = C.c_void_p
        self.lib.rlc_local_cache_stats.argtypes = [C.c_void_p, C.c_void_p]
        self.h = self.lib.rlc_create_fc(size, ratio, 0, 0)
        assert self.h, "HipRateLimitCache (freecache) construction failed"

    def cache_stats(self):
        o = (C.c_uint64 * 6)()
        self.lib.rlc_local_cache_stats(self.h, o)
        return list(o)


class SerialModel:
    """Serial DoLimit: every lookup of a request, then its INCRBYs in order (EXPIRE = divider,
    no jitter), then GetResponseDescriptorStatus per descriptor with the Set of each reply past
    the limit (TTL = divider)."""

    def __init__(self, cache, rules, ratio=0.8):
        self.fc, self.rules, self.ratio = cache, rules, ratio
        self.redis = {}  # key -> [count, expire_at]
        self.stats = [dict(total_hits=0, over_limit=0, near_limit=0, over_limit_with_local_cache=0) for _ in rules]

    def do_limit(self, domain, descs, rules, hits, now):
        h = max(1, hits)
        keys, hit = [], []
        for d, r in zip(descs, rules):
            if r is None:
                keys.append(None)
                hit.append(False)
                continue
            div = hiprl.UNIT_DIVIDER[self.rules[r][1]]
            k = (domain + "_" + "".join(f"{a}_{b}_" for a, b in d) + str(now // div * div)).encode()
            keys.append(k)
            self.stats[r]["total_hits"] += h
            hit.append(self.fc.get(k, now))
        after = [None] * len(descs)
        for i, (k, r) in enumerate(zip(keys, rules)):
            if k is None or hit[i]:
                continue
            c = self.redis.setdefault(k, [0, 0])
            if now >= c[1]:
                c[0] = 0
            c[0] += h
            c[1] = now + hiprl.UNIT_DIVIDER[self.rules[r][1]]
            after[i] = c[0]
        out = []
        for i, (k, r) in enumerate(zip(keys, rules)):
            if k is None:
                out.append((hiprl.CODE_OK, 0, 0, 0))
                continue
            L, unit = self.rules[r]
            div = hiprl.UNIT_DIVIDER[unit]
            st = self.stats[r]
            reset = div - now % div
            if hit[i]:
                st["over_limit"] += h
                st["over_limit_with_local_cache"] += h
                out.append((hiprl.CODE_OVER_LIMIT, 0, 1, reset))
                continue
            a = after[i]
            b = a - h
            near = int(math.floor(float(np.float32(L) * np.float32(self.ratio))))
            if a > L:
                if b >= L:
                    st["over_limit"] += h
                else:
                    st["over_limit"] += a - L
                    st["near_limit"] += L - max(near, b)
                self.fc.set(k, div, now)
                out.append((hiprl.CODE_OVER_LIMIT, 0, 1, reset))
            else:
                if a > near:
                    st["near_limit"] += h if b >= near else a - near
                out.append((hiprl.CODE_OK, L - a, 1, reset))
        return out


def _stream(seed, n_calls, n_keys, rules):
    """Calls of 1..48 descriptors (a few nil, keys Zipf-like over n_keys, duplicates allowed),
    hits 0..3, time advancing 0..2 s every 50 calls (about a minute and a half in all)."""
    rng = np.random.default_rng(seed)
    now = 1_700_000_010
    calls = []
    for c in range(n_calls):
        if c % 50 == 0:
            now += int(rng.integers(0, 3))
        n = int(rng.integers(1, 49))
        ks = np.minimum(rng.zipf(1.3, n) - 1, n_keys - 1) if c % 2 else rng.integers(0, n_keys, n)
        descs = [[("key", f"v{int(k)}")] for k in ks]
        rl = [None if rng.random() < 0.05 else int(k) % len(rules) for k in ks]
        calls.append((descs, rl, int(rng.integers(0, 4)), now))
    return calls


RULES = [(1, hiprl.MINUTE), (2, hiprl.MINUTE), (1, hiprl.HOUR), (4, hiprl.HOUR), (3, hiprl.SECOND)]


def _run(m, model, calls, ids):
    for j, (descs, rl, hits, now) in enumerate(calls):
        m.lib.rlc_set_time(m.h, now)
        got, _ = m.do_limit("fc", descs, [None if r is None else ids[r] for r in rl], hits)
        want = model.do_limit("fc", descs, rl, hits, now)
        assert [tuple(g) for g in got] == want, j
    for r in range(len(RULES)):
        got = m.stats(ids[r])
        for key, v in model.stats[r].items():
            assert got[key] == v, (r, key)


def test_serial_model_matches_the_device_cache():
    """No eviction (a 1-GiB model): the serial model with freecache equals the device's cache."""
    calls = _stream(5, 500, 4000, RULES)
    m = Mirror(True)
    ids = [m.add_rule(L, u, f"r{k}") for k, (L, u) in enumerate(RULES)]
    _run(m, SerialModel(FreeCache(1 << 30), RULES), calls, ids)
    m.close()


@pytest.mark.parametrize("size", [1 << 30, 100])
def test_freecache_batcher_against_serial_model(size):
    """size 1 GiB: nothing evicted (same as the device cache); 100 B (512-KiB floor): about
    11k entries of ~47 B fit and the stream evicts ~2.7k of them, whose keys INCRBY again."""
    calls = _stream(6, 4000, 30000, RULES)
    m = FcMirror(size)
    ids = [m.add_rule(L, u, f"r{k}") for k, (L, u) in enumerate(RULES)]
    model = SerialModel(FreeCache(size), RULES)
    _run(m, model, calls, ids)
    assert m.cache_stats() == model.fc.stats()
    if size == 100:
        assert model.fc.evacuated > 1000 and model.fc.hits > 1000
    m.close()


def test_freecache_batcher_concurrent_callers():
    """8 threads of 300 calls each on keys of their own, sharing batches (2-ms window), a cache
    that does not evict: every thread's statuses equal a serial model of its own calls (a call
    is looked up when enqueued and its Sets are made before it returns), and the per-rule stats
    add up across threads."""
    import threading

    T, n = 8, 300
    m = FcMirror(1 << 30)
    m.lib.rlc_destroy(m.h)
    m.h = m.lib.rlc_create_fc(1 << 30, 0.8, 0, 2000)
    ids = [m.add_rule(L, u, f"r{k}") for k, (L, u) in enumerate(RULES)]
    now = 1_700_000_020
    m.lib.rlc_set_time(m.h, now)
    per = []
    for t in range(T):
        calls = _stream(100 + t, n, 300, RULES)
        per.append([(d, r, h, now) for d, r, h, _ in calls])
    res = [None] * T

    def run(t):
        res[t] = [m.do_limit(f"t{t}", d, [None if x is None else ids[x] for x in r], h)[0] for d, r, h, _ in per[t]]

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    tot = [dict(total_hits=0, over_limit=0, near_limit=0, over_limit_with_local_cache=0) for _ in RULES]
    for t in range(T):
        model = SerialModel(FreeCache(1 << 30), RULES)
        for j, (d, r, h, now_) in enumerate(per[t]):
            assert [tuple(g) for g in res[t][j]] == model.do_limit(f"t{t}", d, r, h, now_), (t, j)
        for k in range(len(RULES)):
            for key, v in model.stats[k].items():
                tot[k][key] += v
    for k in range(len(RULES)):
        got = m.stats(ids[k])
        for key, v in tot[k].items():
            assert got[key] == v, (k, key)
    bs = (C.c_uint64 * 5)()
    m.lib.rlc_batcher_stats.argtypes = [C.c_void_p, C.c_void_p]
    m.lib.rlc_batcher_stats(m.h, bs)
    assert bs[0] < T * n  # calls of several threads shared batches
    m.close()

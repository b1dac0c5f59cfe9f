"""Differential parity: HIP path (C ABI) vs the CPU oracle on seeded request streams.

Bit-exact on every descriptor status, stat delta and request throttle. Streams mix
domains, 1-4 entry descriptors, nil limits, duplicate descriptors in one request,
key-string collisions ("a_b","c" vs "a","b_c"), hits_addend 0..8, per-request limit
overrides sharing one key (different L, same unit), every unit, window rollover, and the
local over-limit cache on and off. (Strings shared by several units: tests/test_per_second.py.)
"""

import numpy as np
import pytest

import hiprl
import oracle
import streams
import workload

pytestmark = pytest.mark.gpu

from streams import LS, RULES, UNITS, batch_sizes, make_stream  # noqa: E402,F401

PIPELINES = ["v4", "lsd"]


def run_both(reqs, sizes, local_cache, sort_bits=48, ratio=0.8, lsd_only=False, pipeline="v4"):
    o = oracle.Oracle(near_limit_ratio=ratio, local_cache=local_cache)
    o.load_rules(RULES)
    e = hiprl.Engine(near_limit_ratio=ratio, local_cache=local_cache, sort_bits=sort_bits, max_batch_desc=1 << 17,
                     lsd_only=lsd_only, pipeline=pipeline)
    e.load_rules(RULES)
    a = streams.replay(o, reqs, sizes)
    b = streams.replay(e, reqs, sizes)
    e.ref_oracle = o
    return a, b, e


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("local_cache", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_streams(seed, local_cache, pipeline):
    reqs = make_stream(seed, 6000, t0=1_700_000_000 - 7 + seed * 3600 * 24 - 130)
    sizes = batch_sizes(reqs, np.random.default_rng(seed + 100), 1500)
    (ost, othr), (gst, gthr), _ = run_both(reqs, sizes, local_cache, pipeline=pipeline)
    streams.assert_same(ost, othr, gst, gthr, f"seed={seed} local={local_cache} pipeline={pipeline}")


@pytest.mark.parametrize("sort_bits", [8, 16, 64])
def test_sort_prefix_widths_and_resort(sort_bits):
    """Narrow sort prefixes make different keys share a sorted run; the LSD pipeline must
    detect it and re-sort on the full fingerprint (resorts > 0 at 8 bits) with identical output."""
    reqs = make_stream(11, 4000, t0=1_600_000_000, keyspace=400)
    sizes = batch_sizes(reqs, np.random.default_rng(5), 2000)
    (ost, othr), (gst, gthr), eng = run_both(reqs, sizes, True, sort_bits=sort_bits, lsd_only=True)
    streams.assert_same(ost, othr, gst, gthr, f"sort_bits={sort_bits}")
    if sort_bits == 8:
        assert eng.stats()["resorts"] > 0


def test_hot_key_long_segments():
    """One key hit thousands of times in one batch (segments span many scan tiles), with
    the local cache freezing it mid-batch, and a second hot key under a large limit."""
    reqs = []
    t = 1_650_000_000
    for i in range(30000):
        if i % 3 == 0:
            reqs.append(("hot", [[("k", "x")]], [2], 1, t))          # L=10 SECOND -> freezes early
        elif i % 3 == 1:
            reqs.append(("hot", [[("k", "y")]], [3 + 4 * 2], 2, t))  # L=40 HOUR
        else:
            reqs.append(("hot", [[("k", f"c{i % 997}")]], [1 + 4], 1, t))
    for lc in (False, True):
        for pl in PIPELINES:
            (ost, othr), (gst, gthr), _ = run_both(reqs, [len(reqs)], lc, pipeline=pl)
            streams.assert_same(ost, othr, gst, gthr, f"hot local={lc} pipeline={pl}")


def hot_stream(n_batches, per_batch, t0, rule_of=None, seed=0):
    """Batches dominated by a few keys (each >= HOT_MIN_SEG per batch, one beyond a 4096
    hot chunk), plus a cold tail; `now` advances 1 s per batch so SECOND keys roll over
    and alternate window parity."""
    rng = np.random.default_rng(seed)
    reqs, sizes = [], []
    for b in range(n_batches):
        t = t0 + b
        for i in range(per_batch):
            x = rng.random()
            if x < 0.45:
                k, r = "h0", 2            # SECOND L=10
            elif x < 0.55:
                k, r = "h1", 3 + 4 * 1    # MINUTE L=40
            elif x < 0.62:
                k, r = f"h{2 + int(rng.integers(0, 6))}", 1 + 4 * 2  # HOUR L=3
            else:
                k, r = f"c{int(rng.integers(0, 5000))}", 3 + 4 * 3   # DAY L=40
            if rule_of is not None:
                r = rule_of(b, k, r)
            reqs.append(("hs", [[("k", k)]], [r], int(rng.integers(0, 4)), t))
        sizes.append(per_batch)
    return reqs, sizes


@pytest.mark.parametrize("local_cache", [False, True])
def test_hot_set_across_batches(local_cache, pipeline="v4"):
    """The v4 pipeline learns hot keys from one batch and gives them their own buckets in
    the next; results stay bit-exact as they roll over windows."""
    reqs, sizes = hot_stream(6, 12000, t0=1_700_000_000 - 3, seed=local_cache)
    (ost, othr), (gst, gthr), eng = run_both(reqs, sizes, local_cache, pipeline=pipeline)
    streams.assert_same(ost, othr, gst, gthr, f"hotset local={local_cache}")
    s = eng.stats()
    assert s["hot_keys"] >= 2, s  # h0, h1 always; h2..h7 hover around HOT_MIN_SEG
    # only the first batch (no hot set yet, one key > 1024 descriptors in an MSD bucket)
    assert s["lsd_fallbacks"] == 1, s
    assert s["inserted_keys"] == eng.ref_oracle.num_strings(), s  # one slot per key string


def test_hot_key_changes_rule(pipeline="v4"):
    """A hot key submitted under a second rule in a later batch sends that batch to the
    LSD pipeline (before anything touches the table); results stay bit-exact."""
    def rule_of(b, k, r):
        return 1 if (b == 3 and k == "h0") else r   # same unit (SECOND), other limit
    reqs, sizes = hot_stream(5, 8000, t0=1_700_000_100, rule_of=rule_of, seed=7)
    (ost, othr), (gst, gthr), eng = run_both(reqs, sizes, True, pipeline=pipeline)
    streams.assert_same(ost, othr, gst, gthr, "hot rule change")
    assert eng.stats()["lsd_fallbacks"] >= 1


def test_oversized_bucket_falls_back():
    """More descriptors than the 2048 MSD buckets hold (1024 each) go to the LSD pipeline."""
    b = workload.config2_batch(0, d=2_400_000, N=3_000_000)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(workload.CONFIG2_RULES)
    e = hiprl.Engine(log2_slots=(23, 12, 12, 12), local_cache=True, max_batch_desc=b.n_desc, max_batch_req=b.n_desc,
                     max_blob_bytes=int(b.blob.shape[0]) + 64)
    e.load_rules(workload.CONFIG2_RULES)
    ost, othr = o.submit(b, threads=8)
    gst, gthr = e.submit(b)
    streams.assert_same(ost, othr, gst, gthr, "oversized bucket")
    assert e.stats()["lsd_fallbacks"] == 1


def test_config3_zipf_batches():
    """The benchmark workload (config 3: 1e8 keys Zipf(1.1), three units) at 1M descriptors
    per batch, three consecutive batches, bit-exact against the oracle."""
    d = 1_000_000
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(workload.CONFIG3_RULES)
    e = hiprl.Engine(log2_slots=(22, 24, 25, 12), local_cache=True, max_batch_desc=d, max_batch_req=d, max_blob_bytes=24 * d)
    e.load_rules(workload.CONFIG3_RULES)
    for k in range(3):
        b = workload.config3_batch(k, d=d)
        ost, othr = o.submit(b, threads=8)
        gst, gthr = e.submit(b)
        streams.assert_same(ost, othr, gst, gthr, f"config3 batch {k}")
    s = e.stats()
    assert s["hot_keys"] > 0 and s["lsd_fallbacks"] == 1, s  # batch 0 learns the hot set


def test_window_rollover_across_batches():
    """Counters reset at each window boundary; old-generation slots are reused."""
    reqs = []
    t = 1_700_003_595  # 5 s before an hour boundary
    for s in range(12):
        for i in range(200):
            reqs.append(("roll", [[("k", str(i % 50))]], [(s + i) % 16], 1 + (i % 3), t + s))
    sizes = [200] * 12
    for lc in (False, True):
        (ost, othr), (gst, gthr), _ = run_both(reqs, sizes, lc)
        streams.assert_same(ost, othr, gst, gthr, f"rollover local={lc}")


def test_large_hits_addend_and_counter_wrap():
    """uint32 wraparound of INCRBY replies (fixed_cache_impl.go:109-110)."""
    big = 0xFFFFFFF0
    reqs = [("w", [[("k", "1")]], [3], big, 1000), ("w", [[("k", "1")]], [3], big, 1000),
            ("w", [[("k", "1")]], [3], 40, 1000), ("w", [[("k", "2")]], [3], 0, 1000)]
    for lc in (False, True):
        (ost, othr), (gst, gthr), _ = run_both(reqs, [2, 2], lc)
        streams.assert_same(ost, othr, gst, gthr, f"wrap local={lc}")


def test_error_paths():
    eng = hiprl.Engine()
    eng.load_rules([(5, hiprl.SECOND)])
    # rule id out of range is rejected before any device work
    with pytest.raises(hiprl.RedisError):
        eng.submit(hiprl.build_batch([("d", [[("a", "b")]], [7], 1, 10)]))
    # a batch spanning three seconds of SECOND windows is rejected
    with pytest.raises(hiprl.RedisError, match="window"):
        eng.submit(hiprl.build_batch([("d", [[("a", "b")]], [0], 1, 10), ("d", [[("a", "b")]], [0], 1, 12)]))
    # the engine keeps working afterwards
    st, _ = eng.submit(hiprl.build_batch([("d", [[("a", "b")]], [0], 1, 13)]))
    assert int(st["limit_remaining"][0]) == 4
    # a region that could pass its load limit refuses the batch before any counter changes
    small = hiprl.Engine(log2_slots=(4, 4, 4, 4))
    small.load_rules([(5, hiprl.SECOND)])
    with pytest.raises(hiprl.RedisError, match="RL_ENOSPC.*load limit"):
        small.submit(hiprl.build_batch([("d", [[("a", str(i))]], [0], 1, 11) for i in range(100)]))
    st, _ = small.submit(hiprl.build_batch([("d", [[("a", "1")]], [0], 1, 11)]))
    assert int(st["limit_remaining"][0]) == 4  # the refused batch left no trace


@pytest.mark.parametrize("which", ["g35", "g43"])
def test_grouping_collisions(which):
    """Two keys whose fingerprints agree on the bucketed pipeline's grouping bits
    (tests/golden/collisions.json), interleaved in one batch: a 35-bit collision is
    regrouped in LDS on wider bits, a 43-bit one by the single-thread stable partition.
    Either way the decisions are bit-exact and the batch stays on the bucketed pipeline."""
    import json
    from pathlib import Path
    c = json.loads((Path(__file__).parent / "golden" / "collisions.json").read_text())
    a, b = c["g35"] if which == "g35" else c["g43"]
    rng = np.random.default_rng(3)
    reqs = []
    for i in range(20000):
        if i % 97 == 0:
            k = a if rng.random() < 0.5 else b
            reqs.append(("coll", [[("k", k)]], [0], int(rng.integers(0, 3)), c["now"]))  # rule 0: L=1 SECOND
        else:
            reqs.append(("cold", [[("k", str(int(rng.integers(0, 50000))))]], [2], 1, c["now"]))
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(RULES)
    e = hiprl.Engine(local_cache=True, max_batch_desc=1 << 15, hash_seed=c["seed"])
    e.load_rules(RULES)
    (ost, othr) = streams.replay(o, reqs)
    (gst, gthr) = streams.replay(e, reqs)
    streams.assert_same(ost, othr, gst, gthr, which)
    assert e.stats()["lsd_fallbacks"] == 0, e.stats()


@pytest.mark.parametrize("L", [500, 3000, 20])
def test_hot_freeze_in_straddling_request(L):
    """v3 and v4 decide hot keys in arrival-order tiles of 2048 descriptors. When the local cache
    freezes a hot key inside a request that continues into later tiles, those later
    descriptors still INCRBY (all lookups of a request precede its Sets,
    fixed_cache_impl.go:55-86); requests after it are local-cache hits. Long requests of
    one hot key start mid-tile and straddle 1-3 tile boundaries."""
    t = 1_700_000_500
    def batch(b, n):
        reqs = []
        rng = np.random.default_rng(b)
        while len(reqs) < n:
            x = rng.random()
            if x < 0.002:
                # one request holding many descriptors of the hot key
                k = int(rng.integers(300, 5000))
                reqs.append(("st", [[("k", "hot")]] * k, [3] * k, 1, t + b))
            elif x < 0.5:
                reqs.append(("st", [[("k", "hot")]], [3], int(rng.integers(0, 3)), t + b))
            else:
                reqs.append(("st", [[("k", f"c{int(rng.integers(0, 3000))}")]], [1], 1, t + b))
        return reqs
    rules = [(L, u) for u in UNITS for L in (1, 3, 10, 40)]
    rules[3] = (L, hiprl.SECOND)  # a new window every batch: the key freezes again in each
    reqs, sizes = [], []
    for b in range(4):
        r = batch(b, 3000)
        reqs += r
        sizes.append(len(r))
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(rules)
    e = hiprl.Engine(near_limit_ratio=0.8, local_cache=True, max_batch_desc=1 << 17)
    e.load_rules(rules)
    a = streams.replay(o, reqs, sizes)
    g = streams.replay(e, reqs, sizes)
    streams.assert_same(*a, *g, f"straddle L={L}")
    assert e.stats()["hot_keys"] >= 1


def _bucket_keys(prefix: str, now: int, n: int = 20000):
    """Key ids whose fingerprints (engine default seed, SECOND unit) share one MSD bucket
    (hi bits 63..53) with different split bits (hi bit 52); also every id's bucket."""
    ids = np.arange(n, dtype=np.uint64)
    blob, off = workload.prefix_blob([prefix.encode() + b"_k_", ids, b"_"])
    hi, _ = oracle.fingerprints(blob, off, now, 0x5EE7AB1E5EED)
    bkt = hi >> np.uint64(53)
    half = (hi >> np.uint64(52)) & np.uint64(1)
    for i in range(n):
        same = np.nonzero((bkt == bkt[i]) & (half != half[i]))[0]
        if len(same):
            return int(i), int(same[0]), bkt
    raise AssertionError("no split pair")


@pytest.mark.parametrize("local_cache", [False, True])
def test_v4_oversized_bucket_paths(local_cache):
    """v4 groups each MSD range in LDS (at most 640 records). A larger bucket of a first
    batch (no hot set yet) is split by the fingerprint bit below the bucket bits into two
    halves of whole keys (keys a, b: ~480 descriptors each, same bucket, different halves);
    a half still too large (key c: ~800 descriptors) is grouped in the block's global
    scratch. Bit-exact either way, and the batch stays on the v4 pipeline."""
    now = 1_700_000_100
    a, b, bkt = _bucket_keys("sp", now)
    c = next(i for i in range(len(bkt)) if bkt[i] != bkt[a])
    rng = np.random.default_rng(11)
    reqs = []
    for i in range(8000):
        x = rng.random()
        if x < 0.06:
            k = a
        elif x < 0.12:
            k = b
        elif x < 0.22:
            k = c
        else:
            k = 20000 + int(rng.integers(0, 3000))
        reqs.append(("sp", [[("k", str(k))]], [2], int(rng.integers(0, 3)), now))  # SECOND L=10
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=local_cache)
    o.load_rules(RULES)
    e = hiprl.Engine(near_limit_ratio=0.8, local_cache=local_cache, max_batch_desc=1 << 14, pipeline="v4")
    e.load_rules(RULES)
    g = streams.replay(e, reqs, [len(reqs)])
    ref = streams.replay(o, reqs, [len(reqs)])
    streams.assert_same(*ref, *g, f"v4 oversized local={local_cache}")
    assert e.stats()["lsd_fallbacks"] == 0, e.stats()

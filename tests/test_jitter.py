"""EXPIRATION_JITTER_MAX_SECONDS (VERDICT r4 missing 4 / next 6).

The reference adds JitterRand.Int63n(max) to every EXPIRE (src/redis/fixed_cache_impl.go:69-72;
default max 300, src/settings/settings.go:43): a key lives until its last INCRBY's now +
divider + that INCRBY's jitter. The draws are made by the host batcher in serial (enqueue) order
and travel with the batch (rl_batch.ttl_jitter, one per descriptor); the device applies exactly
the EXPIRE of each key's last INCRBY. The jitter shows in decisions where a key string is shared
by units of different sizes: a SECOND key at a minute-aligned second is the MINUTE window's key
string, so whether a MINUTE request 20 s later continues the counter depends on the SECOND
INCRBY's jitter.

CPU: the oracle against TestRedisWithJitter (test/redis/fixed_cache_impl_test.go:451-479:
Int63 -> 100, max 3600 -> EXPIRE 101) and hand-derived shared-string sequences. GPU: both
pipelines, the hot-key path (with and without local-cache freezes), the compact host format, the
routed path and the C++ batcher, bit-exact against the oracle given the same draws. With the
local cache on the reference skips the draw for a local-cache hit, which the batcher cannot know
before the device decides: there every descriptor with a limit gets a draw (the same
distribution, another assignment of values to keys); with it off (the default) the assignment is
the reference's.
"""
import numpy as np
import pytest
import torch  # noqa: F401  (initialised before the engines, as in the other GPU test modules)

import hiprl
import oracle
from streams import assert_same, batch_sizes

T0 = 1_699_920_000  # a multiple of 86400
S, M = 0, 1
RULES = [(10, hiprl.SECOND), (600, hiprl.MINUTE)]


def go_int63n(int63_draws, n):
    """Go math/rand (*Rand).Int63n(n) over a source's successive Int63() values."""
    if n & (n - 1) == 0:
        return next(int63_draws) & (n - 1)
    mx = (1 << 63) - 1 - (1 << 63) % n
    v = next(int63_draws)
    while v > mx:
        v = next(int63_draws)
    return v % n


def one(rule, t, h=1, key=("key", "value"), dom="domain"):
    return (dom, [[key]], [rule], h, t)


def run_oracle(reqs, jit, local_cache=False, rules=RULES):
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(rules)
    outs = []
    d = 0
    for r in reqs:
        n = len(r[1])
        b = hiprl.build_batch([r], jit=jit[d:d + n])
        outs.append(o.submit(b))
        d += n
    return o, outs


def test_redis_with_jitter_vector():
    """TestRedisWithJitter: SECOND limit 10 at 1234, INCRBY -> 5, jitter source Int63 -> 100 with
    max 3600: EXPIRE 101, status OK 5. Replayed as five INCRBYs of the key, the fifth with the
    draw: the key lives until 1234 + 101."""
    j = go_int63n(iter([100]), 3600)
    assert j == 100
    reqs = [one(0, 1234)] * 5
    o, outs = run_oracle(reqs, [0, 0, 0, 0, j])
    st = outs[-1][0]
    assert int(st["code_flags"][0]) & 0xFF == hiprl.CODE_OK and int(st["limit_remaining"][0]) == 5
    key = b"domain_key_value_1234"
    assert o.counter(key, 1234 + 100) == 5
    assert o.counter(key, 1234 + 101) == -1
    # without the draw the key is gone one second later
    o0, _ = run_oracle(reqs, [0] * 5)
    assert o0.counter(key, 1235) == -1


def test_jitter_keeps_shared_string_alive():
    """A SECOND INCRBY at a minute-aligned second then a MINUTE request 20 s later: with a
    jitter above 19 the MINUTE request continues the counter (post-value 2), otherwise the key
    expired and it starts over (post-value 1). The last INCRBY's jitter decides."""
    for jit_s, want in ((0, 599), (19, 599), (20, 598), (300, 598)):
        _, outs = run_oracle([one(S, T0), one(M, T0 + 20)], [jit_s, 0])
        assert int(outs[1][0]["limit_remaining"][0]) == want, (jit_s, want)
    # two SECOND INCRBYs: the second one's EXPIRE wins (30 then 5: expired at T0 + 20)
    _, outs = run_oracle([one(S, T0), one(S, T0), one(M, T0 + 20)], [30, 5, 0])
    assert int(outs[2][0]["limit_remaining"][0]) == 599
    _, outs = run_oracle([one(S, T0), one(S, T0), one(M, T0 + 20)], [5, 30, 0])
    assert int(outs[2][0]["limit_remaining"][0]) == 597


def jitter_stream(seed, n_req=3000, t0=T0 - 2, jmax=40):
    """Requests around aligned windows (strings shared by units), every descriptor with a
    jitter draw: time moves 0-1 s every ~20 requests, sometimes a window ahead."""
    rng = np.random.default_rng(seed)
    reqs, jit, t = [], [], t0
    rules4 = [(5, hiprl.SECOND), (40, hiprl.MINUTE), (90, hiprl.HOUR), (200, hiprl.DAY)]
    for _ in range(n_req):
        if rng.random() < 0.05:
            t += int(rng.integers(0, 2)) + (int(rng.integers(5, 40)) if rng.random() < 0.03 else 0)
        descs, rules = [], []
        for _ in range(int(rng.integers(1, 4))):
            descs.append([("k", f"v{int(rng.integers(0, 4))}")])
            rules.append(int(rng.choice(4, p=[0.4, 0.3, 0.2, 0.1])))
            jit.append(int(rng.integers(0, jmax)))
        reqs.append(("dom", descs, rules, int(rng.integers(0, 4)), t))
    return rules4, reqs, np.array(jit, np.uint16)


def batches_of(reqs, jit, sizes):
    out, i, d = [], 0, 0
    for n in sizes:
        part = reqs[i:i + n]
        nd = sum(len(r[1]) for r in part)
        out.append(hiprl.build_batch(part, jit=jit[d:d + nd]))
        i += n
        d += nd
    return out


def test_oracle_jitter_stream_batch_split_invariant():
    rules, reqs, jit = jitter_stream(3, 1500)
    res = []
    for sizes in (batch_sizes(reqs, np.random.default_rng(2), 10 ** 6), batch_sizes(reqs, np.random.default_rng(1), 60)):
        o = oracle.Oracle()
        o.load_rules(rules)
        outs = [o.submit(b) for b in batches_of(reqs, jit, sizes)]
        res.append((np.concatenate([x[0] for x in outs]), np.concatenate([x[1] for x in outs])))
    assert_same(*res[0], *res[1])
    # the jitter changes this stream's decisions (it is not a no-op input)
    o = oracle.Oracle()
    o.load_rules(rules)
    outs = [o.submit(b) for b in batches_of(reqs, np.zeros_like(jit), batch_sizes(reqs, np.random.default_rng(2), 10 ** 6))]
    assert not np.array_equal(np.concatenate([x[0] for x in outs]), res[0][0])


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["v4", "lsd"])
@pytest.mark.parametrize("local_cache", [False, True])
def test_gpu_jitter_same_string_stream(pipeline, local_cache):
    rules, reqs, jit = jitter_stream(5 + local_cache, 4000)
    sizes = batch_sizes(reqs, np.random.default_rng(7), 300)
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(rules)
    e = hiprl.Engine(local_cache=local_cache, pipeline=pipeline)
    e.load_rules(rules)
    for k, b in enumerate(batches_of(reqs, jit, sizes)):
        assert_same(*e.submit(b), *o.submit(b), ctx=f"{pipeline} lc={local_cache} batch={k}")


@pytest.mark.gpu
def test_gpu_jitter_compact_format():
    """rl_batch_c.ttl_jitter: the compact host format (the batchers' default) carries the draws."""
    rules, reqs, jit = jitter_stream(9, 3000)
    sizes = batch_sizes(reqs, np.random.default_rng(8), 400)
    o = oracle.Oracle()
    o.load_rules(rules)
    e = hiprl.Engine()
    e.load_rules(rules)
    for k, b in enumerate(batches_of(reqs, jit, sizes)):
        assert_same(*e.submit_compact(b), *o.submit(b), ctx=f"compact batch={k}")


def hot_stream(local_cache, seed):
    """Hot keys on the v4 hot path: 4 prefixes with 600 SECOND descriptors each per batch for
    10 seconds before T0 (the hot set forms), then a batch at T0 (minute-aligned) whose
    descriptors carry jitters 0..40, then a batch at T0 + 20 with each prefix once under the
    MINUTE rule (a second rule for a hot prefix: that batch reruns on the LSD pipeline, which
    reads the EXPIRE the hot path wrote). With the local cache (limit 300) the keys freeze
    mid-batch: the EXPIRE is the freezing request's last INCRBY's."""
    rng = np.random.default_rng(seed)
    L = 300 if local_cache else 100_000
    rules = [(L, hiprl.SECOND), (L, hiprl.MINUTE)]
    batches = []
    for t in [T0 - 10 + k for k in range(10)] + [T0]:
        reqs, jit = [], []
        for q in range(2400 + 200):
            if q < 2400:
                key = f"h{q % 4}"
                nd = 1 + int(rng.random() < 0.1)  # some requests hold a duplicate
            else:
                key = f"c{int(rng.integers(0, 5000))}"
                nd = 1
            reqs.append(("hot", [[("k", key)]] * nd, [S] * nd, 1, t))
            jit += [int(rng.integers(0, 41)) if t == T0 else 0 for _ in range(nd)]
        batches.append(hiprl.build_batch(reqs, jit=jit))
    batches.append(hiprl.build_batch([("hot", [[("k", f"h{k}")]], [M], 1, T0 + 20) for k in range(4)],
                                     jit=[0] * 4))
    return rules, batches


@pytest.mark.gpu
@pytest.mark.parametrize("local_cache", [False, True])
def test_gpu_jitter_hot_keys(local_cache):
    for seed in range(4):
        rules, batches = hot_stream(local_cache, seed)
        o = oracle.Oracle(local_cache=local_cache)
        o.load_rules(rules)
        e = hiprl.Engine(local_cache=local_cache, max_batch_desc=8192)
        e.load_rules(rules)
        fb = []
        for k, b in enumerate(batches):
            f0 = e.stats()["lsd_fallbacks"]
            assert_same(*e.submit(b), *o.submit(b), ctx=f"lc={local_cache} seed={seed} batch={k}")
            fb.append(e.stats()["lsd_fallbacks"] - f0)
        assert e.stats()["hot_keys"] >= 4
        assert fb[-2] == 0 and fb[-1] == 1, fb  # T0 on the hot path; T0 + 20 on the LSD pipeline


@pytest.mark.gpu
def test_gpu_jitter_routed_emulated():
    """The routed path: each record carries its descriptor's jitter to the owner (combining is
    off for a batch with jitter). G = 3 emulated ranks, the same-string stream cut per origin."""
    from test_gpu_emulated_router import drive, parallel

    from test_gpu_combining import check  # noqa: F401 (same checker shape)
    import routing
    G = 3
    rules, reqs, jit = jitter_stream(11, 7200)
    per = 200
    steps, i, d = [], 0, 0
    while i + G * per <= len(reqs):
        row = []
        t = T0 - 8 + 4 * len(steps)  # one time per step, 4 s apart: EXPIREs with small jitter lapse
        for _ in range(G):
            part = [(dm, de, ru, h, t) for (dm, de, ru, h, _) in reqs[i:i + per]]
            nd = sum(len(r[1]) for r in part)
            row.append(hiprl.build_batch(part, jit=jit[d:d + nd]))
            i += per
            d += nd
        steps.append(row)

    class Ranks:
        pass
    ranks = Ranks()
    ranks.G = G
    wid = hiprl.Router.emu_world(G)
    ranks.engines = []
    for _ in range(G):
        e = hiprl.Engine(max_batch_desc=3 * per * G * 3, max_batch_req=3 * per * G * 3)
        e.load_rules(rules)
        ranks.engines.append(e)
    ranks.routers = [None] * G
    parallel(G, lambda r: ranks.routers.__setitem__(r, hiprl.Router([ranks.engines[r]], max_desc=3 * per, n_shards=G,
                                                                     rank=r, rccl_id=wid, emulated=True)))
    bufs, codes = drive(ranks, steps, "pipelined")
    o = oracle.Oracle()
    o.load_rules(rules)
    for s, (row, bf) in enumerate(zip(steps, bufs)):
        assert all(codes[r][s] is None for r in range(G)), codes
        est, ethr = o.submit(routing.concat_batches(row))
        d0 = r0 = 0
        for g, (b, (gst, gthr)) in enumerate(zip(row, bf.results())):
            assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], gst, gthr, f"routed step={s} origin={g}")
            d0 += b.n_desc
            r0 += b.n_req
    assert ranks.routers[0].stats()["combined_steps"] == 0
    parallel(G, lambda r: ranks.routers[r].close())
    torch.cuda.synchronize()

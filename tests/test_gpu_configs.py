"""BASELINE configs 1 and 2 on the default v4 path, a window that holds many batches with the
table regions well filled, capacity refusal, and the host (PCIe) submit path — all bit-exact
against the CPU oracle (the serial DoLimit restatement, oracle/rl_oracle.cpp).

Reference semantics: `src/redis/fixed_cache_impl.go:31-123` over a Redis whose keys live for
their window (EXPIRE div, `:69-72`); test shapes follow `test/redis/fixed_cache_impl_test.go`
at the §8(d) config sizes.
"""
import numpy as np
import pytest
import torch

import hiprl
import oracle
import streams
import workload
from test_gpu_pipelined import _oracle, _pipelined

pytestmark = pytest.mark.gpu


def _engine(rules, local_cache, d, log2, blob, **kw):
    e = hiprl.Engine(log2_slots=log2, local_cache=local_cache, max_batch_desc=d, max_batch_req=d,
                     max_blob_bytes=blob, **kw)
    e.load_rules(rules)
    return e


@pytest.mark.parametrize("local_cache", [False, True])
def test_config2_uniform_1m_batches(local_cache):
    """Config 2: 1e6 uniform keys, SECOND L=5, 1e6-descriptor batches, three consecutive
    batches (now + 1 s each) on v4 with no fallback."""
    d = 1_000_000
    bs = [workload.config2_batch(k, d=d) for k in range(3)]
    e = _engine(workload.CONFIG2_RULES, local_cache, d, (22, 12, 12, 12), 24 * d)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=local_cache)
    o.load_rules(workload.CONFIG2_RULES)
    for k, b in enumerate(bs):
        ost, othr = o.submit(b, threads=8)
        gst, gthr = e.submit(b)
        streams.assert_same(ost, othr, gst, gthr, f"config2 batch {k} lc={local_cache}")
    s = e.stats()
    assert s["lsd_fallbacks"] == 0 and s["batches"] == 3, s
    assert s["inserted_keys"] == o.num_strings(), s


def test_config2_pipelined_depth2():
    """Config 2 with two batches in flight (rl_submit_pipelined), local cache on."""
    d = 1_000_000
    bs = [workload.config2_batch(k, d=d) for k in range(4)]
    e = _engine(workload.CONFIG2_RULES, True, d, (22, 12, 12, 12), 24 * d)
    got = _pipelined(e, bs, torch.device("cuda", 0), depth=2)
    want = _oracle(bs, workload.CONFIG2_RULES, True)
    streams.assert_same(*want, *got, "config2 pipelined")
    assert e.stats()["lsd_fallbacks"] == 0


@pytest.mark.parametrize("local_cache", [False, True])
def test_config1_examples_ratelimit(local_cache):
    """Config 1: examples/ratelimit rules (rl.foo.baz SECOND 1, mongo_cps SECOND 500), 10k keys."""
    e = _engine(workload.CONFIG1_RULES, local_cache, 10_000, (16, 12, 12, 12), 64 * 10_000)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=local_cache)
    o.load_rules(workload.CONFIG1_RULES)
    for k in range(4):
        b = workload.config1_batch(k)
        streams.assert_same(*o.submit(b), *e.submit(b), f"config1 batch {k}")
    assert e.stats()["lsd_fallbacks"] == 0


def _live_stream(n_batches, per_batch, t0, keys_per_unit, seed, roll_at):
    """Batches of one-descriptor requests, uniform over keys_per_unit keys of each of three
    units; `now` stays t0 for roll_at batches (one window holds them all), then t0 + 1."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        t = t0 + (b >= roll_at)
        rule = rng.integers(0, 3, per_batch).astype(np.uint32)
        key = rng.integers(0, keys_per_unit, per_batch).astype(np.uint64) * np.uint64(3) + rule.astype(np.uint64)
        blob, off = workload.prefix_blob([b"live_k_", key, b"_"])
        h = rng.integers(0, 3, per_batch).astype(np.uint32)
        out.append(hiprl.Batch(blob, off, rule, np.arange(per_batch, dtype=np.uint32),
                               np.full(per_batch, t, np.int64), h))
    return out


@pytest.mark.parametrize("pipeline", ["v4", "lsd"])
def test_window_of_64_batches_fills_regions(pipeline):
    """One SECOND window holds 64 batches (as at 8000 batches/s a real window holds
    thousands): the SECOND / MINUTE / HOUR regions end above half full, probe chains get
    long, and every decision stays bit-exact; then the second rolls over and the SECOND
    region's new generation starts empty."""
    rules = [(40, hiprl.SECOND), (300, hiprl.MINUTE), (1000, hiprl.HOUR)]
    t0 = 1_700_000_021  # SECOND / MINUTE / HOUR keys each in their own home region
    bs = _live_stream(72, 2000, t0, 10_000, 5, roll_at=64)
    e = _engine(rules, True, 2000, (14, 14, 14, 12), 64 * 2000, pipeline=pipeline)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=True)
    o.load_rules(rules)
    fill = None
    for k, b in enumerate(bs):
        streams.assert_same(*o.submit(b), *e.submit(b), f"live batch {k}")
        if k == 63:
            occ = e.occupancy()
            fill = [occ["live"][r] / occ["slots"][r] for r in range(8) if occ["live"][r]]
    assert len(fill) == 3 and min(fill) >= 0.5, fill  # S, M, H regions of the window
    occ = e.occupancy()
    s_regions = [r for r in (0, 1) if occ["live"][r]]
    assert len(s_regions) == 2 and min(occ["live"][r] for r in s_regions) < 0.5 * occ["slots"][0], occ
    assert e.stats()["inserted_keys"] == o.num_strings()


@pytest.mark.parametrize("pipeline", ["v4", "lsd"])
def test_capacity_refusal_changes_nothing(pipeline):
    """A batch that could push a region past its load limit is refused (RL_ENOSPC) before any
    counter changes: the next batch decides exactly as if the refused one never came."""
    rules = [(3, hiprl.SECOND)]
    t = 1_700_000_021
    def batch(ids, h=1):
        return hiprl.build_batch([("cap", [[("k", str(i))]], [0], h, t) for i in ids])
    e = _engine(rules, True, 4096, (10, 10, 10, 10), 64 * 4096, pipeline=pipeline)  # limit 768 slots
    o = oracle.Oracle(local_cache=True)
    o.load_rules(rules)
    # the check is conservative: a region's live slots + the batch's descriptors in it
    ok1, refused, ok2 = batch(range(500)), batch(range(500, 900), 2), batch(range(300, 550))
    streams.assert_same(*o.submit(ok1), *e.submit(ok1), "first")
    with pytest.raises(hiprl.RedisError, match="RL_ENOSPC"):
        e.submit(refused)
    assert e.occupancy()["live"][0] + e.occupancy()["live"][1] == 500
    streams.assert_same(*o.submit(ok2), *e.submit(ok2), "after refusal")


@pytest.mark.parametrize("local_cache", [False, True])
def test_host_path_three_in_flight_and_staged(local_cache):
    """rl_submit of host batches with three in flight (H2D, kernels and D2H of different batches
    overlap), results copied out by rl_wait_into; and a batch built in place in a staging slot
    (rl_host_acquire, no host copy). Bit-exact against the serial oracle."""
    reqs = streams.make_stream(21, 9000, t0=1_700_000_000 - 40)
    sizes = streams.batch_sizes(reqs, np.random.default_rng(3), 1200)
    hbs, i = [], 0
    for n in sizes:
        hbs.append(hiprl.build_batch(reqs[i:i + n]))
        i += n
    e = hiprl.Engine(local_cache=local_cache, max_batch_desc=1 << 14)
    e.load_rules(streams.RULES)
    got, pend = [], []
    for k, b in enumerate(hbs):
        if k % 4 == 3:  # built in place in the slot
            sl = e.host_acquire()
            nb = int(b.blob.shape[0])
            sl["blob"][:nb] = b.blob
            sl["off"][:b.n_desc + 1] = b.off
            sl["rule"][:b.n_desc] = b.rule
            sl["req_of"][:b.n_desc] = b.req_of
            sl["now"][:b.n_req] = b.now
            sl["hits"][:b.n_req] = b.hits
            e.submit_staged(b.n_desc, b.n_req, nb, sl)
        else:
            e.submit_host_async(b)
        pend.append(b)
        if len(pend) == hiprl.MAX_IN_FLIGHT:
            got.append(_collect(e, pend[0], k))
            pend.pop(0)
    for j, b in enumerate(pend):
        got.append(_collect(e, b, j))
    want = _oracle(hbs, streams.RULES, local_cache)
    streams.assert_same(*want, np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]), "host path")
    assert e.stats()["host_batches"] == len(hbs)


def _collect(e, b, k):
    """Every other batch through rl_wait_view (results read in the pinned slot, copied here
    before the next submit reuses it), the others through rl_wait_into."""
    if k % 2:
        st, thr = e.wait_view(b.n_desc, b.n_req)
        return st.copy(), thr.copy()
    return e.wait_into(b.n_desc, b.n_req)


def test_wait_view_refuses_device_batches():
    """rl_wait_view only hands out a host batch's slot: on a device batch it gives RL_ESTATE,
    completes nothing, and rl_wait still completes that batch."""
    import router

    dev = torch.device("cuda", 0)
    reqs = [("wv", [[("k", str(i % 11))]], [0], 1, 1_700_000_000) for i in range(200)]
    hb = hiprl.build_batch(reqs)
    db = router.DeviceBatch.from_host(hb, dev)
    out = torch.zeros(200 * 20, dtype=torch.uint8, device=dev)
    thr = torch.zeros(200, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    e = hiprl.Engine(max_batch_desc=1 << 10)
    e.load_rules(streams.RULES)
    e.submit_device_async(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), out.data_ptr(), thr.data_ptr())
    with pytest.raises(hiprl.RedisError):
        e.wait_view(hb.n_desc, hb.n_req)
    e.wait()
    # a host batch submitted with nothing in flight: its view equals the oracle's answer
    e.submit_host_async(hb)
    st, th = e.wait_view(hb.n_desc, hb.n_req)
    o = oracle.Oracle()
    o.load_rules(streams.RULES)
    o.submit(hb)  # the device batch above decided the same requests first
    ost, oth = o.submit(hb)
    streams.assert_same(ost, oth, st.copy(), th.copy(), "wait_view")

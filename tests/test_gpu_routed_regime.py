"""The routed regime a multi-GPU scaling run measures, checked against the oracle at size
(VERDICT r4 weak 1 / next 2a).

G = 8 ranks over the router's collective transport (emulated in process: the RCCL transport's
code with its three collectives as device copies driven by the same count and displacement
vectors), BASELINE config 3 traffic — 1e8 keys, Zipf s = 1.1, SECOND / MINUTE / HOUR rules by
rank % 3 — at 1e5 descriptors per origin batch, each origin its own stream (the bench's seeds),
2^24-slot regions per rank, combining on, 32 steps (four route hot-set refreshes, so hot keys
travel as one combined record per origin), two steps per simulated second and origins 0-2 s
apart inside a step. Every step must equal one serial DoLimit stream over the origins' batches in
rank order: oracle.submit(threads=16) over the rank-order concatenation, every status, stat delta
and request ThrottleMillis. Reference: src/redis/fixed_cache_impl.go:31-123 (INCRBY per key in
serial order), src/redis/driver_impl.go:84-110 (each key's commands to the node owning it).
"""
import numpy as np
import pytest
import torch

import hiprl
import oracle
import routing
import streams
import workload
from test_gpu_combining import Bufs
from test_gpu_emulated_router import drive, parallel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
T0 = 1_700_000_020


class Ranks:
    def __init__(self, G, per, log2=24, local_cache=False):
        self.G = G
        wid = hiprl.Router.emu_world(G)
        cap = per * G
        self.engines = []
        for _ in range(G):
            e = hiprl.Engine(log2_slots=(log2, log2, log2, 12), max_batch_desc=cap, max_batch_req=cap,
                             max_blob_bytes=cap * 24 + 64, local_cache=local_cache)
            e.load_rules(workload.CONFIG3_RULES)
            self.engines.append(e)
        self.routers = [None] * G

        def mk(r):
            self.routers[r] = hiprl.Router([self.engines[r]], max_desc=per, n_shards=G, rank=r, rccl_id=wid,
                                           emulated=True)
        parallel(G, mk)

    def close(self):
        parallel(self.G, lambda r: self.routers[r].close())


def config3_steps(G, steps, per, seed=19):
    rng = np.random.default_rng(seed)
    out = []
    for s in range(steps):
        row = []
        for g in range(G):
            b = workload.config3_batch(s, d=per, seed=3 + 7919 * g, t0=T0)
            t = T0 + s // 2 + int(rng.integers(0, 3))  # origins 0-2 s apart inside a step
            row.append(hiprl.Batch(b.blob, b.off, b.rule, b.req_of, np.full(b.n_req, t, np.int64), b.hits))
        out.append(row)
    return out


@pytest.mark.parametrize("local_cache", [False, True])
def test_routed_config3_g8_full_regime_against_oracle(local_cache):
    """Combining on (local cache off): hot keys as one record per origin. With the local cache
    on (no combining: a freeze inside a group needs the per-descriptor sequence) the SECOND keys
    of the hot set pass L = 10 within a step and every later request is a local-cache hit."""
    G, steps, per = 8, (32 if not local_cache else 16), 100_000
    rows = config3_steps(G, steps, per)
    ranks = Ranks(G, per, local_cache=local_cache)
    bufs, codes = drive(ranks, rows, "pipelined", depth=3)
    assert all(c is None for cr in codes for c in cr), codes
    st = [r.stats() for r in ranks.routers]
    assert all(x["status"] == [0] * G and x["steps"] == steps for x in st), st
    assert len({x["step_clock"] for x in st}) == 1
    routed = G * per
    recv = sum(r.stats()["recv"][i] for i, r in enumerate(ranks.routers))
    if local_cache:
        assert st[0]["combined_steps"] == 0 and recv == routed, (st[0], recv)
    else:
        assert st[0]["combined_steps"] >= steps // 2 and st[0]["hot_groups"] > 0, st[0]
        assert recv < 0.75 * routed, (recv, routed)  # combined hot records
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(workload.CONFIG3_RULES)
    for s, (row, bf) in enumerate(zip(rows, bufs)):
        est, ethr = o.submit(routing.concat_batches(row), threads=16)
        d0 = r0 = 0
        for g, (b, (gst, gthr)) in enumerate(zip(row, bf.results())):
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], gst, gthr, f"step={s} origin={g}")
            d0 += b.n_desc
            r0 += b.n_req
    occ = [e.occupancy() for e in ranks.engines]
    assert sum(sum(x["live"]) for x in occ) > 0
    ranks.close()


def test_routed_config5_g4_rollover_against_oracle():
    """BASELINE config 5 routed: G = 4 emulated ranks, Zipf(1.1) keys over 10⁸ with SECOND /
    MINUTE / HOUR rules by rank % 3 and hits_addend ~ U{1..8}, 10⁵ descriptors per origin, one
    step per simulated second for 24 s across a minute boundary (window rollover and expiry on
    the owners), origins 0-2 s apart, combining on. Every status and ThrottleMillis against one
    serial oracle over the rank-order concatenation."""
    G, steps, per = 4, 24, 100_000
    rng = np.random.default_rng(5)
    t0 = 1_700_000_000 - 37
    rows = []
    for s in range(steps):
        row = []
        for g in range(G):
            b = workload.config5_batch(s, d=per, N=100_000_000, batches_per_s=1, seed=5 + 7919 * g, t0=t0)
            t = t0 + s + int(rng.integers(0, 3))
            row.append(hiprl.Batch(b.blob, b.off, b.rule, b.req_of, np.full(b.n_req, t, np.int64), b.hits))
        rows.append(row)
    wid = hiprl.Router.emu_world(G)
    engines = []
    for _ in range(G):
        e = hiprl.Engine(log2_slots=(22, 22, 22, 12), max_batch_desc=per * G, max_batch_req=per * G,
                         max_blob_bytes=per * G * 24 + 64)
        e.load_rules(workload.CONFIG5_RULES)
        engines.append(e)
    routers = [None] * G

    def mk(r):
        routers[r] = hiprl.Router([engines[r]], max_desc=per, n_shards=G, rank=r, rccl_id=wid, emulated=True)
    parallel(G, mk)

    class R:
        pass
    ranks = R()
    ranks.G, ranks.routers = G, routers
    bufs, codes = drive(ranks, rows, "pipelined", depth=3)
    assert all(c is None for cr in codes for c in cr), codes
    st = [r.stats() for r in routers]
    assert all(x["status"] == [0] * G and x["steps"] == steps for x in st), st
    o = oracle.Oracle(near_limit_ratio=0.8)
    o.load_rules(workload.CONFIG5_RULES)
    for s, (row, bf) in enumerate(zip(rows, bufs)):
        est, ethr = o.submit(routing.concat_batches(row), threads=16)
        d0 = r0 = 0
        for g, (b, (gst, gthr)) in enumerate(zip(row, bf.results())):
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], gst, gthr, f"step={s} origin={g}")
            d0 += b.n_desc
            r0 += b.n_req
    parallel(G, lambda r: routers[r].close())

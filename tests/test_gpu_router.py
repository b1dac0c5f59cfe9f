"""Routed (multi-shard) decisions through the C ABI on one GPU vs the serial CPU oracle.

G engines on cuda:0 stand in for G GPUs: each packs its own batch with rl_route_pack, the
all-to-alls are done by slicing (tests/routing.exchange_local), every owner decides what it
receives with rl_submit_routed, and each origin unpacks with rl_route_unpack. The outputs
must equal one oracle replaying the origins' batches in rank order — bit-exact statuses,
stat deltas and ThrottleMillis — for the v4 and LSD pipelines, local cache on and off, a
skewed stream whose hot keys go through v4 hot buckets, and empty shards.
"""
import numpy as np
import pytest
import torch

import hiprl
import oracle
import routing
import router
import streams

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def make_shards(G, local_cache, pipeline, cap=1 << 15):
    shards = []
    for g in range(G):
        e = hiprl.Engine(local_cache=local_cache, max_batch_desc=cap, pipeline=pipeline)
        e.load_rules(streams.RULES)
        shards.append(router.EngineShard(e, g, G, DEV, cap))
    return shards


def run_routed(G, steps_batches, local_cache, pipeline):
    """steps_batches[s][g] = origin g's host batch of step s; returns per-step outputs."""
    shards = make_shards(G, local_cache, pipeline)
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(streams.RULES)
    for s, batches in enumerate(steps_batches):
        dbs = [router.DeviceBatch.from_host(b, DEV) for b in batches]
        outs, counts = routing.exchange_local(shards, dbs)
        torch.cuda.synchronize()
        est, ethr = o.submit(routing.concat_batches(batches))
        d0 = r0 = 0
        for g, b in enumerate(batches):
            st = outs[g][0].cpu().numpy().view(hiprl.STATUS_DTYPE)
            thr = outs[g][1].cpu().numpy().view(np.uint32)
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], st, thr,
                                f"G={G} step={s} origin={g} pipeline={pipeline} local={local_cache}")
            # the device partition is the restated one
            own = routing.owners_of(b, streams.RULES, G, 0x5EE7AB1E5EED)
            assert counts[g] == [int((own == j).sum()) for j in range(G)]
            d0 += b.n_desc
            r0 += b.n_req
    return shards


def stream_batches(G, steps, per, seed, keyspace=30):
    out = []
    for s in range(steps):
        row = []
        for g in range(G):
            reqs = streams.make_stream(seed + 17 * g + 1000 * s, per, t0=1_700_000_000 + s, keyspace=keyspace,
                                       dt_max=1)
            reqs = [(d, de, ru, h, 1_700_000_000 + s) for d, de, ru, h, _ in reqs]
            row.append(hiprl.build_batch(reqs))
        out.append(row)
    return out


@pytest.mark.parametrize("pipeline", ["v4", "lsd"])
@pytest.mark.parametrize("local_cache", [False, True])
@pytest.mark.parametrize("G", [2, 4])
def test_routed_random_streams(G, local_cache, pipeline):
    run_routed(G, stream_batches(G, 4, 1500, seed=G), local_cache, pipeline)


@pytest.mark.parametrize("pipeline", ["v4"])
def test_routed_hot_keys(pipeline):
    """A few keys take most descriptors on every origin: the owners' hot sets form from
    routed candidates and later steps decide those keys in v4's hot buckets."""
    G, steps = 3, 12
    rng = np.random.default_rng(3)
    out = []
    for s in range(steps):
        row = []
        for g in range(G):
            reqs = []
            for i in range(4000):
                x = rng.random()
                key = f"h{int(rng.integers(0, 4))}" if x < 0.6 else f"c{int(rng.integers(0, 5000))}"
                rule = 4 * 0 + 3 if key.startswith("h") else 4 + 2  # SECOND L=40 / MINUTE L=10
                reqs.append(("hot", [[("k", key)]], [rule], int(rng.integers(0, 3)), 1_700_000_000 + s))
            row.append(hiprl.build_batch(reqs))
        out.append(row)
    for lc in (False, True):
        shards = run_routed(G, out, lc, pipeline)
        assert max(sh.eng.stats()["hot_keys"] for sh in shards) > 0


def test_routed_empty_and_nil_only():
    """Origins with no descriptors, nil limits only, and owners that receive nothing."""
    G = 3
    nil = hiprl.NIL_RULE
    b_empty = hiprl.build_batch([])
    b_nil = hiprl.build_batch([("d", [[("k", "v")], [("k", "w")]], [nil, nil], 1, 1_700_000_000)])
    b_one = hiprl.build_batch([("d", [[("k", "v")]], [1], 2, 1_700_000_000)])
    run_routed(G, [[b_empty, b_nil, b_one], [b_one, b_empty, b_empty], [b_nil, b_nil, b_nil]], True, "v4")

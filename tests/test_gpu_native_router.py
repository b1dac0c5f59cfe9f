"""The routed step owned by the C ABI (rl_router_*, csrc/rl_router.cpp) vs the serial oracle.

Local transport: G engines on cuda:0 stand in for G GPUs (exchanges by device copies).
RCCL transport: a one-rank communicator on cuda:0 (the collectives run for real, each rank
sending to itself). Decisions must equal one oracle replaying the origins' batches in shard
order, bit-exact. Error steps: a bad batch on one origin and an owner that cannot take its
records make every shard's step fail (its own code or RL_EPEER), and the router keeps working.
Reference: src/redis/fixed_cache_impl.go:31-123 per key on the server that owns it
(driver_impl.go:84-110 pipelines per server).
"""
import numpy as np
import pytest
import torch

import hiprl
import oracle
import router
import routing
import streams
from test_gpu_router import DEV, stream_batches

pytestmark = pytest.mark.gpu


def _engines(G, local_cache, cap):
    es = []
    for _ in range(G):
        e = hiprl.Engine(local_cache=local_cache, max_batch_desc=cap)
        e.load_rules(streams.RULES)
        es.append(e)
    return es


def _step(r, batches):
    dbs = [router.DeviceBatch.from_host(b, DEV) for b in batches]
    outs = [torch.empty(max(1, b.n_desc) * 20, dtype=torch.uint8, device=DEV) for b in batches]
    thrs = [torch.empty(max(1, b.n_req), dtype=torch.int32, device=DEV) for b in batches]
    torch.cuda.synchronize()
    r.step([hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs()) for db in dbs],
           [o.data_ptr() for o in outs], [t.data_ptr() for t in thrs])
    return [(o.cpu().numpy().view(hiprl.STATUS_DTYPE)[:b.n_desc], t.cpu().numpy().view(np.uint32)[:b.n_req])
            for o, t, b in zip(outs, thrs, batches)]


def _check(o, batches, got, ctx):
    est, ethr = o.submit(routing.concat_batches(batches))
    d0 = r0 = 0
    for g, (b, (st, thr)) in enumerate(zip(batches, got)):
        streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], st, thr, f"{ctx} origin={g}")
        d0 += b.n_desc
        r0 += b.n_req


@pytest.mark.parametrize("local_cache", [False, True])
@pytest.mark.parametrize("G", [1, 3, 4])
def test_local_transport_matches_serial_oracle(G, local_cache):
    per = 1500  # requests per origin batch (1-3 descriptors each)
    es = _engines(G, local_cache, 4 * per * G)
    r = hiprl.Router(es, max_desc=4 * per)
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(streams.RULES)
    for s, batches in enumerate(stream_batches(G, 4, per, seed=40 + G)):
        got = _step(r, batches)
        _check(o, batches, got, f"G={G} step={s}")
        st = r.stats()
        routed = sum(int((b.rule != hiprl.NIL_RULE).sum()) for b in batches)
        assert sum(st["recv"]) == routed and st["status"] == [0] * G, st
        own0 = routing.owners_of(batches[0], streams.RULES, G, 0x5EE7AB1E5EED)
        assert st["sent"] == [int((own0 == j).sum()) for j in range(G)]


def test_rccl_transport_one_rank(monkeypatch):
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    per = 1500
    es = _engines(1, True, 4 * per)
    r = hiprl.Router(es, max_desc=4 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    o = oracle.Oracle(local_cache=True)
    o.load_rules(streams.RULES)
    for s, batches in enumerate(stream_batches(1, 3, per, seed=9)):
        _check(o, batches, _step(r, batches), f"rccl step={s}")
    assert r.stats()["steps"] == 3
    r.close()


def test_local_transport_errors_fail_every_shard():
    G, per = 3, 1000
    es = _engines(G, True, 4 * per * G)
    r = hiprl.Router(es, max_desc=4 * per)
    o = oracle.Oracle(local_cache=True)
    o.load_rules(streams.RULES)
    steps = stream_batches(G, 3, per, seed=77)
    _check(o, steps[0], _step(r, steps[0]), "before")
    bad = list(steps[1])
    b1 = bad[1]
    rule = b1.rule.copy()
    rule[len(rule) // 2] = 99  # unknown rule id on origin 1
    bad[1] = hiprl.Batch(b1.blob, b1.off, rule, b1.req_of, b1.now, b1.hits)
    with pytest.raises(hiprl.RedisError, match="shard 1 \\(pack\\)") as ex:
        _step(r, bad)
    assert ex.value.code == -1 and r.stats()["status"][1] == -1
    # the failed step changed nothing: the next one equals the oracle without it
    _check(o, steps[2], _step(r, steps[2]), "after")


def test_owner_over_capacity_fails_every_shard():
    """Owner 1 can decide at most 2000 records; both origins send it more (requests picked so
    that all their descriptors route to shard 1): the step fails on both shards."""
    G, per = 2, 1500
    batches = []
    for g in range(G):
        reqs = [(d, de, ru, h, 1_700_000_000) for d, de, ru, h, _ in
                streams.make_stream(300 + g, 4000, t0=1_700_000_000, keyspace=400, dt_max=1)]
        b = hiprl.build_batch(reqs)
        own = routing.owners_of(b, streams.RULES, G, 0x5EE7AB1E5EED)
        to1 = np.ones(b.n_req, bool)
        np.logical_and.at(to1, b.req_of, own != 0)
        keep = [q for q in range(b.n_req) if to1[q]]
        sel, n = [], 0
        for q in keep:
            n += len(reqs[q][1])
            if n > per:
                break
            sel.append(reqs[q])
        batches.append(hiprl.build_batch(sel))
    assert all(600 < b.n_desc <= per for b in batches)
    es = [hiprl.Engine(local_cache=True, max_batch_desc=c) for c in (per * G, 2000)]
    for e in es:
        e.load_rules(streams.RULES)
    r = hiprl.Router(es, max_desc=per)
    with pytest.raises(hiprl.RedisError, match="shard 1 \\(decide\\)") as ex:
        _step(r, batches)
    assert ex.value.code == -4 and r.stats()["status"] == [-7, -4], r.stats()  # the other shard: RL_EPEER


def test_rccl_transport_one_rank_errors(monkeypatch):
    """RCCL transport error steps: a batch the device finds malformed (unknown rule id: the
    pack's status rides in the counts exchange) and a batch over max_desc (found on the host)
    (an owner that cannot take its records is covered on the local transport above: at one
    rank the pack's capacity check comes first) fail the step with the shard's own code, and the
    router keeps working: the next step equals the oracle without the failed ones."""
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    per = 1200
    e = hiprl.Engine(local_cache=True, max_batch_desc=4 * per)
    e.load_rules(streams.RULES)
    r = hiprl.Router([e], max_desc=4 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    o = oracle.Oracle(local_cache=True)
    o.load_rules(streams.RULES)
    steps = stream_batches(1, 3, per, seed=31)
    _check(o, steps[0], _step(r, steps[0]), "before")
    b = steps[1][0]
    rule = b.rule.copy()
    rule[len(rule) // 3] = 77
    with pytest.raises(hiprl.RedisError, match="shard 0 \\(pack\\)") as ex:
        _step(r, [hiprl.Batch(b.blob, b.off, rule, b.req_of, b.now, b.hits)])
    assert ex.value.code == -1 and r.stats()["status"][0] == -1
    big = routing.concat_batches(stream_batches(1, 5, per, seed=32)[0] * 5)
    assert big.n_desc > 4 * per
    with pytest.raises(hiprl.RedisError, match="shard 0 \\(pack\\)") as ex:
        _step(r, [big])
    assert ex.value.code == -4
    _check(o, steps[2], _step(r, steps[2]), "after")
    r.close()


def test_rccl_transport_stall_times_out(monkeypatch):
    """VERDICT r5 next-3a on the RCCL transport itself (one-rank communicator): the exchange
    stream held before the counts exchange (RL_ROUTER_FAULT=stall:0). The bounded host wait
    polls ncclCommGetAsyncError, gives up after RL_ROUTER_TIMEOUT_MS, aborts the communicator
    (ncclCommAbort) and returns RL_ECOMM; every later call fails the same way and destroy
    completes (the stalled kernel is released by the abort)."""
    import time
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    monkeypatch.setenv("RL_ROUTER_FAULT", "stall:0")
    monkeypatch.setenv("RL_ROUTER_TIMEOUT_MS", "1500")
    per = 1000
    e = hiprl.Engine(local_cache=True, max_batch_desc=4 * per)
    e.load_rules(streams.RULES)
    r = hiprl.Router([e], max_desc=4 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    monkeypatch.delenv("RL_ROUTER_FAULT")
    monkeypatch.delenv("RL_ROUTER_TIMEOUT_MS")
    steps = stream_batches(1, 2, per, seed=33)
    t0 = time.monotonic()
    with pytest.raises(hiprl.RedisError, match="no progress within 1500 ms") as ex:
        _step(r, steps[0])
    assert ex.value.code == -8 and time.monotonic() - t0 < 15
    with pytest.raises(hiprl.RedisError) as ex2:
        _step(r, steps[1])
    assert ex2.value.code == -8
    r.close()
    o = oracle.Oracle(local_cache=True)
    o.load_rules(streams.RULES)
    b = steps[1][0]
    gs, gt = e.submit(b)
    es_, et = o.submit(b)
    streams.assert_same(es_, et, gs, gt, "engine after the stalled router")


def test_router_refuses_an_engine_that_decided_batches_without_the_lag_window():
    """a router's engines keep the previous SECOND generation live (lag window); an
    engine that already decided batches under the one-generation rule would under-count its
    live slots in lag mode, so rl_router_create refuses it (RL_ESTATE) and leaves it as it was;
    the same engine created with RL_CFG_LAG_WINDOW serves a router after deciding batches."""
    for lag in (False, True):
        e = hiprl.Engine(local_cache=False, max_batch_desc=4000, lag_window=lag)
        e.load_rules(streams.RULES)
        b = stream_batches(1, 1, 800, seed=41)[0][0]
        e.submit(b)
        if lag:
            r = hiprl.Router([e], max_desc=4000)
            r.close()
            continue
        with pytest.raises(hiprl.RedisError) as ex:
            hiprl.Router([e], max_desc=4000)
        assert ex.value.code == -5  # RL_ESTATE
        o = oracle.Oracle()
        o.load_rules(streams.RULES)
        o.submit(b)
        b2 = stream_batches(1, 1, 800, seed=42)[0][0]
        gs, gt = e.submit(b2)
        es, et = o.submit(b2)
        streams.assert_same(es, et, gs, gt, "engine after the refused router")

"""The combining router (csrc/rl_router.cpp + the k_route_pack2 / k_route_hot_scan /
k_route_unpack_raw kernels of csrc/rl_route.hip) vs the serial oracle, bit-exact.

An origin sends the descriptors of a hot prefix (its route hot set, refreshed every 8 steps
from the owners' hot sets) as ONE record carrying their sum of hits_addend; owners answer every
record with its raw INCRBY post-value and origins rebuild each descriptor's post-value and make
the decision. Every step must equal one oracle replaying the origins' batches in shard order —
statuses, stat deltas, ThrottleMillis — through the local transport (G logical shards on one
GPU), a one-rank RCCL communicator, two steps in flight, and the host-memory entry. Batches a
combined record cannot represent exactly (two request times among hot descriptors, a hot prefix
under a second rule, a huge hits_addend) are packed again without combining (the repack). The
local cache on disables combining. Fault injection (RL_ROUTER_FAULT) checks that every shard
leaves a failed step together and that the router keeps working.
Reference: src/redis/fixed_cache_impl.go:31-123 (INCRBY per key in serial order, decisions per
descriptor) with the key's counter on its owner, src/redis/driver_impl.go:84-110.
"""
import numpy as np
import pytest
import torch

import hiprl
import oracle
import router
import routing
import streams
import workload

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
SEED = 0x5EE7AB1E5EED
# streams.RULES plus their shadow-mode twins (ids 16..31; an extension, rl_hip.h RL_RULE_SHADOW)
RULES = list(streams.RULES) + [(L, u, True) for (L, u) in streams.RULES]


def skew_batches(G, steps, per, seed, hot_keys=6, hot_p=0.55, t0=1_700_000_000, dup_p=0.05, h_max=8):
    """Per step and origin `per` requests: hot_p of them on a few hot keys (one rule each, some
    shadow), the rest on 20000 cold keys; 1-2 descriptors, duplicates inside a request,
    h in 0..h_max; every request of a step at one time (t0 + step)."""
    rng = np.random.default_rng(seed)
    hot_rule = [int(rng.integers(0, len(RULES))) for _ in range(hot_keys)]
    out = []
    for s in range(steps):
        row = []
        for g in range(G):
            reqs = []
            for _ in range(per):
                nd = 1 + int(rng.random() < 0.2)
                descs, rules = [], []
                for _ in range(nd):
                    if rng.random() < hot_p:
                        k = int(rng.integers(0, hot_keys))
                        descs.append([("hot", f"h{k}")])
                        rules.append(hot_rule[k])
                    else:
                        k = int(rng.integers(0, 20000))
                        descs.append([("c", str(k))])
                        rules.append(k % len(RULES))
                if rng.random() < dup_p:
                    descs.append(descs[0])
                    rules.append(rules[0])
                reqs.append(("cmb", descs, rules, int(rng.integers(0, h_max + 1)), t0 + s))
            row.append(hiprl.build_batch(reqs))
        out.append(row)
    return out


def engines(G, cap, local_cache=False, rules=RULES, pipeline="v4", log2_slots=(16, 16, 16, 14), blob=0):
    es = []
    for _ in range(G):
        e = hiprl.Engine(local_cache=local_cache, max_batch_desc=cap, max_batch_req=cap, pipeline=pipeline,
                         log2_slots=log2_slots, max_blob_bytes=blob or None)
        e.load_rules(rules)
        es.append(e)
    return es


class Bufs:
    def __init__(self, batches):
        self.dbs = [router.DeviceBatch.from_host(b, DEV) for b in batches]
        self.outs = [torch.zeros(max(1, b.n_desc) * 20, dtype=torch.uint8, device=DEV) for b in batches]
        self.thrs = [torch.zeros(max(1, b.n_req), dtype=torch.int32, device=DEV) for b in batches]
        self.batches = batches

    def args(self):
        return ([hiprl.Engine.device_batch(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs()) for db in self.dbs],
                [o.data_ptr() for o in self.outs], [t.data_ptr() for t in self.thrs])

    def results(self):
        torch.cuda.synchronize()
        return [(o.cpu().numpy().view(hiprl.STATUS_DTYPE)[:b.n_desc], t.cpu().numpy().view(np.uint32)[:b.n_req])
                for o, t, b in zip(self.outs, self.thrs, self.batches)]


def check(o, batches, got, ctx):
    est, ethr = o.submit(routing.concat_batches(batches))
    d0 = r0 = 0
    for g, (b, (st, thr)) in enumerate(zip(batches, got)):
        streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], st, thr, f"{ctx} origin={g}")
        d0 += b.n_desc
        r0 += b.n_req


def run_steps(r, steps, o, mode="sync", ctx="", depth=2):
    """Every step through the router (sync: step; pipelined: `depth` in flight; host: submit_host /
    wait_into), each checked against the oracle in order."""
    if mode == "host":
        for s, batches in enumerate(steps):
            r.submit_host(batches)
            got = r.wait_into([(b.n_desc, b.n_req) for b in batches])
            check(o, batches, got, f"{ctx} step={s}")
        return
    if mode == "sync":
        for s, batches in enumerate(steps):
            bf = Bufs(batches)
            torch.cuda.synchronize()
            r.step(*bf.args())
            check(o, batches, bf.results(), f"{ctx} step={s}")
        return
    pend = []
    for s, batches in enumerate(steps):
        bf = Bufs(batches)
        torch.cuda.synchronize()
        r.submit(*bf.args())
        pend.append((s, bf))
        if len(pend) == depth:
            s0, b0 = pend.pop(0)
            r.wait()
            check(o, b0.batches, b0.results(), f"{ctx} step={s0}")
    for s0, b0 in pend:
        r.wait()
        check(o, b0.batches, b0.results(), f"{ctx} step={s0}")


def new_oracle(local_cache=False):
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(RULES)
    return o


@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_combining_local_transport(G):
    per = 2500
    steps = skew_batches(G, 18, per, seed=100 + G)
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per)
    run_steps(r, steps, new_oracle(), "sync", f"local G={G}")
    st = r.stats()
    assert st["combined_steps"] >= 6 and st["hot_groups"] > 0, st
    assert st["status"] == [0] * G
    # the hot descriptors travelled as one record per group: owners decided fewer records
    routed = sum(int((b.rule != hiprl.NIL_RULE).sum()) for b in steps[-1])
    assert sum(st["recv"]) < 0.7 * routed, (sum(st["recv"]), routed)
    r.close()


def test_combining_rccl_one_rank_two_in_flight(monkeypatch):
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    per = 3000
    steps = skew_batches(1, 20, per, seed=7)
    r = hiprl.Router(engines(1, 3 * per), max_desc=3 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    run_steps(r, steps, new_oracle(), "pipelined", "rccl")
    st = r.stats()
    assert st["combined_steps"] >= 6 and st["steps"] == 20, st
    r.close()


def test_combining_rccl_one_rank_three_in_flight(monkeypatch):
    """Three steps in flight (bench.py's default): every submit exchanges the replies of the two
    older steps after its counts, and their unpacks follow its records."""
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    per = 3000
    steps = skew_batches(1, 20, per, seed=9)
    r = hiprl.Router(engines(1, 3 * per), max_desc=3 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    run_steps(r, steps, new_oracle(), "pipelined", "rccl depth 3", depth=3)
    st = r.stats()
    assert st["combined_steps"] >= 6 and st["steps"] == 20, st
    r.close()


def test_combining_local_two_in_flight():
    G, per = 3, 2000
    steps = skew_batches(G, 16, per, seed=17)
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per)
    run_steps(r, steps, new_oracle(), "pipelined", "local pipelined")
    assert r.stats()["combined_steps"] >= 4
    r.close()


def test_repack_when_a_group_is_not_one_key_string():
    """After the hot set forms: a step whose hot descriptors carry two request times, one where
    a hot prefix arrives under a second rule, one with hits_addend past the combining range.
    Each is packed again without combining (repacks) and stays bit-exact."""
    G, per = 2, 2000
    steps = skew_batches(G, 12, per, seed=23)
    tail = skew_batches(G, 6, per, seed=24, t0=1_700_000_012)
    # (a) two times: the second half of origin 0's requests one second later
    b = tail[0][0]
    now = b.now.copy()
    now[b.n_req // 2:] += 1
    tail[0][0] = hiprl.Batch(b.blob, b.off, b.rule, b.req_of, now, b.hits)
    # (b) a second rule on a hot prefix: rewrite one hot descriptor's rule
    b = tail[2][1]
    rule = b.rule.copy()
    hot_i = [i for i in range(b.n_desc) if b.prefix(i).startswith(b"cmb_hot_")]
    rule[hot_i[len(hot_i) // 2]] = (int(rule[hot_i[len(hot_i) // 2]]) + 1) % len(RULES)
    tail[2][1] = hiprl.Batch(b.blob, b.off, rule, b.req_of, b.now, b.hits)
    # (c) a huge hits_addend on a request with a hot descriptor
    b = tail[4][0]
    hits = b.hits.copy()
    hits[int(b.req_of[[i for i in range(b.n_desc) if b.prefix(i).startswith(b"cmb_hot_")][0]])] = 100_000
    tail[4][0] = hiprl.Batch(b.blob, b.off, b.rule, b.req_of, b.now, hits)
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per)
    run_steps(r, steps + tail, new_oracle(), "sync", "repack")
    st = r.stats()
    assert st["repacks"] >= 2 and st["combined_steps"] >= 3, st
    r.close()


def test_repack_over_many_pack_blocks():
    """A repack over many pack blocks: a batch of ~75k descriptors (74 pack blocks of 1024, the
    repack's look-back over all of them) whose hot descriptors carry two request times, after the
    hot set formed; then a big step that combines. Bit-exact against the oracle."""
    G, per, big = 2, 2000, 60_000
    steps = skew_batches(G, 12, per, seed=31)
    tail = skew_batches(G, 2, big, seed=32, t0=1_700_000_012)
    b = tail[0][0]
    now = b.now.copy()
    now[b.n_req // 2:] += 1
    tail[0][0] = hiprl.Batch(b.blob, b.off, b.rule, b.req_of, now, b.hits)
    cap = max(b.n_desc for row in tail for b in row)
    assert cap > 64 * 1024, cap
    r = hiprl.Router(engines(G, cap * G, log2_slots=(20, 20, 20, 20)), max_desc=cap)
    run_steps(r, steps + tail, new_oracle(), "sync", "repack many blocks")
    st = r.stats()
    assert st["repacks"] >= 1 and st["combined_steps"] >= 3, st
    r.close()


def test_local_cache_never_combines():
    G, per = 2, 2000
    steps = skew_batches(G, 12, per, seed=31)
    r = hiprl.Router(engines(G, 3 * per * G, local_cache=True), max_desc=3 * per)
    run_steps(r, steps, new_oracle(local_cache=True), "sync", "local cache")
    assert r.stats()["combined_steps"] == 0
    r.close()


def test_no_combine_flag_and_lsd_engines():
    G, per = 2, 1500
    steps = skew_batches(G, 10, per, seed=37)
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per, combine=False)
    run_steps(r, steps, new_oracle(), "pipelined", "no combine")
    assert r.stats()["combined_steps"] == 0
    r.close()
    r = hiprl.Router(engines(G, 3 * per * G, pipeline="lsd"), max_desc=3 * per)
    run_steps(r, skew_batches(G, 10, per, seed=38), new_oracle(), "pipelined", "lsd engines")
    r.close()


@pytest.mark.parametrize("transport", ["local", "rccl"])
def test_host_memory_entry(transport, monkeypatch):
    """rl_router_submit_host / rl_router_wait_into (a Go service's batch from host memory) and
    rl_router_host_acquire (built in the router's pinned slot): bit-exact, combining on."""
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    G = 4 if transport == "local" else 1
    per = 2000
    steps = skew_batches(G, 12, per, seed=41)
    kw = dict(n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id()) if transport == "rccl" else {}
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per, host=True, max_blob_bytes=3 * per * 24, **kw)
    o = new_oracle()
    run_steps(r, steps[:10], o, "host", transport)
    # the last steps built in place in the pinned slots
    for s, batches in enumerate(steps[10:]):
        slots = []
        for g, b in enumerate(batches):
            sl = r.host_acquire(g)
            n = int(b.blob.shape[0])
            sl["blob"][:n] = b.blob
            sl["off"][:b.n_desc + 1] = b.off
            sl["rule"][:b.n_desc] = b.rule
            sl["req_of"][:b.n_desc] = b.req_of
            sl["now"][:b.n_req] = b.now
            sl["hits"][:b.n_req] = b.hits
            slots.append(dict(sl, n_desc=b.n_desc, n_req=b.n_req, blob_bytes=n))
        r.submit_host(slots)
        check(o, batches, r.wait_into([(b.n_desc, b.n_req) for b in batches]), f"{transport} acquired step={s}")
    assert r.stats()["combined_steps"] >= 2
    r.close()


@pytest.mark.parametrize("phase", ["pack", "records", "decide", "replies", "unpack"])
def test_fault_injection_local_every_shard_returns(phase, monkeypatch):
    """A HIP failure injected on shard 2 of 4 at each phase: the step fails with that shard's
    code (RL_EHIP) and every other shard's status says RL_EPEER (an unpack failure, after the
    last exchange, only loses shard 2's own results); the next steps equal the oracle."""
    G, per = 4, 1200
    steps = skew_batches(G, 4, per, seed=53)
    monkeypatch.setenv("RL_ROUTER_FAULT", f"{phase}:2")
    r = hiprl.Router(engines(G, 3 * per * G), max_desc=3 * per)
    monkeypatch.delenv("RL_ROUTER_FAULT")
    o = new_oracle()
    bf = Bufs(steps[0])
    torch.cuda.synchronize()
    with pytest.raises(hiprl.RedisError, match=f"shard 2 \\({phase}\\)") as ex:
        r.step(*bf.args())
    assert ex.value.code == -2
    st = r.stats()
    assert st["status"][2] == -2 and all(st["status"][j] == -7 for j in range(G) if j != 2), st
    # what the owners applied (per-shard atomicity): nothing after a pack failure; all but owner
    # 2's keys when owner 2 never decided (records); everything when the failure came after the
    # decisions (decide, replies, unpack)
    if phase == "records":
        part = []
        for b in steps[0]:
            own = routing.owners_of(b, RULES, G, SEED)
            rule = np.where(own == 2, hiprl.NIL_RULE, b.rule).astype(np.uint32)
            part.append(hiprl.Batch(b.blob, b.off, rule, b.req_of, b.now, b.hits))
        o.submit(routing.concat_batches(part))
    elif phase != "pack":
        o.submit(routing.concat_batches(steps[0]))
    run_steps(r, steps[1:], o, "sync", f"after {phase} fault")
    r.close()


@pytest.mark.parametrize("phase", ["pack", "records", "decide", "replies", "unpack"])
def test_fault_injection_rccl_one_rank(phase, monkeypatch):
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    per = 1200
    steps = skew_batches(1, 4, per, seed=59)
    monkeypatch.setenv("RL_ROUTER_FAULT", f"{phase}:0")
    r = hiprl.Router(engines(1, 3 * per), max_desc=3 * per, n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id())
    monkeypatch.delenv("RL_ROUTER_FAULT")
    o = new_oracle()
    bf = Bufs(steps[0])
    torch.cuda.synchronize()
    with pytest.raises(hiprl.RedisError, match=f"shard 0 \\({phase}\\)") as ex:
        r.step(*bf.args())
    assert ex.value.code == -2 and r.stats()["status"][0] == -2
    if phase != "pack" and phase != "records":
        o.submit(routing.concat_batches(steps[0]))
    run_steps(r, steps[1:], o, "sync", f"rccl after {phase} fault")
    r.close()


def test_strided_pack_large_grid():
    """3e6 descriptors in one origin batch: 2930 pack blocks (several times what is resident at
    once), the look-back across them, combining on — bit-exact against the oracle; and the
    one-kernel pack of rl_route_pack_strided at 1.2e6 (4688 blocks of 256) equals the
    three-kernel pack."""
    n = 3_000_000
    b = workload.config3_batch(5, d=n)
    e = engines(1, n, rules=workload.CONFIG3_RULES, log2_slots=(22, 22, 22, 12), blob=int(b.blob.shape[0]) + 64)
    r = hiprl.Router(e, max_desc=n)
    o = oracle.Oracle()
    o.load_rules(workload.CONFIG3_RULES)
    bf = Bufs([b])
    torch.cuda.synchronize()
    r.step(*bf.args())
    est, ethr = o.submit(b, threads=8)
    st, thr = bf.results()[0]
    streams.assert_same(est, ethr, st, thr, "3e6 descriptors")
    r.close()
    # rl_route_pack_strided vs rl_route_pack at 1.2e6 descriptors, 4 owners
    m = 1_200_000
    b2 = workload.config3_batch(6, d=m)
    eng = hiprl.Engine(max_batch_desc=m, max_batch_req=m, max_blob_bytes=int(b2.blob.shape[0]) + 64)
    eng.load_rules(workload.CONFIG3_RULES)
    db = router.DeviceBatch.from_host(b2, DEV)
    G = 4
    send_a = torch.zeros(m * 32, dtype=torch.uint8, device=DEV)
    perm_a = torch.zeros(m, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(16, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    counts = eng.route_pack(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), 0, G, send_a.data_ptr(), cnt.data_ptr(),
                            perm_a.data_ptr())
    send_b = torch.zeros(G * m * 32, dtype=torch.uint8, device=DEV)
    perm_b = torch.zeros(m, dtype=torch.int32, device=DEV)
    x = torch.zeros(2 * G, dtype=torch.int32, device=DEV)
    eng.route_pack_strided(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), 0, G, m, send_b.data_ptr(), x.data_ptr(),
                           perm_b.data_ptr())
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    assert list(xs[0::2]) == counts and list(xs[1::2]) == [0] * G
    sa = send_a.cpu().numpy().view(routing.REC_DTYPE)
    sb = send_b.cpu().numpy().view(routing.REC_DTYPE).reshape(G, m)
    off = np.concatenate([[0], np.cumsum(counts)])
    for j in range(G):
        assert np.array_equal(sa[off[j]:off[j + 1]], sb[j, :counts[j]]), j
    pa = perm_a.cpu().numpy().view(np.uint32)
    pb = perm_b.cpu().numpy().view(np.uint32)
    own = pb // m
    assert np.array_equal(pa, np.array([off[o] + p % m for o, p in zip(own, pb)], np.uint32))


@pytest.mark.parametrize("transport", ["local8", "rccl1"])
def test_config4_stream_routed(transport, monkeypatch):
    """BASELINE config 4's stream (device-resolved 4-entry descriptors, half the rules in shadow
    mode, local cache on: no combining) through 8 local shards and a one-rank RCCL router."""
    import config_oracle  # noqa: F401  (the oracle's GetLimit is checked in test_gpu_resolve)
    import rl_config

    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    y = workload.config4_yaml(4)
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    rules = [(r[0], r[1], k % 2 == 0) for k, r in enumerate(cfg.rule_table())]
    G = 8 if transport == "local8" else 1
    es = []
    for _ in range(G):
        e = hiprl.Engine(local_cache=True, max_batch_desc=8000 * G, max_batch_req=8000 * G)
        cfg.install(e)
        e.load_rules(rules)
        es.append(e)
    kw = dict(n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id()) if G == 1 else {}
    r = hiprl.Router(es, max_desc=8000, **kw)
    o = oracle.Oracle(local_cache=True)
    o.load_rules(rules)
    rng = np.random.default_rng(44)
    steps = []
    for s in range(6):
        row = []
        for g in range(G):
            descs = workload.config4_descriptors(1000 + 10 * s + g, 4000, values=40)
            rid = es[0].resolve(rl_config.ResolveBatch([(d, e, None) for d, e in descs]))
            reqs, i = [], 0
            while i < len(descs):
                k = int(rng.integers(1, 5))
                grp = list(range(i, min(i + k, len(descs))))
                reqs.append((descs[grp[0]][0], [descs[j][1] for j in grp], [int(rid[j]) for j in grp],
                             int(rng.integers(0, 9)), 1_700_000_000 + s))
                i += k
            row.append(hiprl.build_batch(reqs))
        steps.append(row)
    run_steps(r, steps, o, "pipelined", f"config4 {transport}")
    r.close()


@pytest.mark.parametrize("transport", ["local8", "rccl1"])
def test_config5_stream_routed(transport, monkeypatch):
    """BASELINE config 5's stream (75 simulated seconds, SECOND/MINUTE/HOUR windows rolling
    over, h ~ U{1..8}, near-limit stats) through 8 local shards and a one-rank RCCL router with
    two steps in flight, combining on."""
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    G = 8 if transport == "local8" else 1
    per = 1500
    es = engines(G, per * G, rules=workload.CONFIG5_RULES)
    kw = dict(n_shards=1, rank=0, rccl_id=hiprl.Router.unique_id()) if G == 1 else {}
    r = hiprl.Router(es, max_desc=per, **kw)
    o = oracle.Oracle()
    o.load_rules(workload.CONFIG5_RULES)
    steps = [[workload.config5_batch(s * G + g, per, 3000, batches_per_s=2, seed=5 + g) for g in range(G)]
             for s in range(150)]
    # every origin of a step at the same time (the stream's clock), 2 steps per second
    steps = [[hiprl.Batch(b.blob, b.off, b.rule, b.req_of, np.full(b.n_req, 1_700_000_000 - 37 + s // 2, np.int64),
                          b.hits) for b in row] for s, row in enumerate(steps)]
    run_steps(r, steps, o, "pipelined", f"config5 {transport}")
    assert r.stats()["combined_steps"] > 0
    r.close()


def test_lookback_spin_expiry_reports_edevice_everywhere(monkeypatch):
    """The packs' decoupled look-back with its spin bound at 0 (RL_DIAG_LB_SPIN_LIMIT, read by
    rl_create): blocks that find a predecessor unpublished give up at once. Every owner's
    (count, status) pair must then carry RL_EDEVICE — one status per origin, so every rank
    leaves the step at the counts exchange — and the router step fails with RL_EDEVICE
    ("device fault"), for the one-kernel pack (k_route_pack1, 256 descriptors per block) and the
    combining router's pack (1024 per block), on grids far larger than what is resident."""
    n = 2_000_000
    b = workload.config3_batch(9, d=n)
    monkeypatch.setenv("RL_DIAG_LB_SPIN_LIMIT", "0")
    e = engines(1, n, rules=workload.CONFIG3_RULES, log2_slots=(22, 22, 22, 12), blob=int(b.blob.shape[0]) + 64)[0]
    monkeypatch.delenv("RL_DIAG_LB_SPIN_LIMIT")
    db = router.DeviceBatch.from_host(b, DEV)
    G = 4
    send = torch.zeros(G * n * 32, dtype=torch.uint8, device=DEV)
    perm = torch.zeros(n, dtype=torch.int32, device=DEV)
    x = torch.zeros(2 * G, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    e.route_pack_strided(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), 0, G, n, send.data_ptr(), x.data_ptr(),
                         perm.data_ptr())
    torch.cuda.synchronize()
    st = x.cpu().numpy()[1::2]
    assert len(set(st.tolist())) == 1, st  # one status for every owner
    assert st[0] == -6, st
    r = hiprl.Router([e], max_desc=n)
    bf = Bufs([b])
    torch.cuda.synchronize()
    with pytest.raises(hiprl.RedisError, match="device fault") as ex:
        r.step(*bf.args())
    assert ex.value.code == -6
    r.close()
    # a fresh engine restores the bound: the same batch packs cleanly
    e2 = engines(1, n, rules=workload.CONFIG3_RULES, log2_slots=(22, 22, 22, 12), blob=int(b.blob.shape[0]) + 64)[0]
    x.zero_()
    e2.route_pack_strided(db.n_desc, db.n_req, db.blob_bytes(), db.ptrs(), 0, G, n, send.data_ptr(), x.data_ptr(),
                          perm.data_ptr())
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    assert list(xs[1::2]) == [0] * G and int(xs[0::2].sum()) == n


@pytest.mark.parametrize("combine", [True, False])
def test_refused_owner_leaves_the_others_decided(combine):
    """Owner 1 cannot take its records (engine capacity 1000): the step fails with its
    RL_ECAPACITY on shard 1 and RL_EPEER on shard 0, but every descriptor owner 0 decided has
    its decision in the outputs (equal to an oracle that applies only owner 0's keys) and owner
    1's descriptors come out RL_CODE_UNKNOWN; the next steps see only what was applied."""
    G, per = 2, 1500
    steps = skew_batches(G, 12, per, seed=61)
    es = engines(1, 3 * per * G) + engines(1, 3 * per * G)
    r = hiprl.Router(es, max_desc=3 * per, combine=combine)
    o = new_oracle()
    run_steps(r, steps[:10], o, "sync", "before")
    small = hiprl.Engine(max_batch_desc=1000, max_batch_req=1000)
    small.load_rules(RULES)
    # owner 1's engine replaced by one too small: a router over (engine 0, small engine) that
    # shares engine 0's table; owner 1's table is empty, so only owner 0's decisions are checked
    r2 = hiprl.Router([es[0], small], max_desc=3 * per, combine=combine)
    bf = Bufs(steps[10])
    torch.cuda.synchronize()
    with pytest.raises(hiprl.RedisError, match="shard 1 \\(decide\\)") as ex:
        r2.step(*bf.args())
    assert ex.value.code == -4 and r2.stats()["status"] == [-7, -4], r2.stats()
    got = bf.results()
    part = []
    for b in steps[10]:
        own = routing.owners_of(b, RULES, G, SEED)
        part.append(hiprl.Batch(b.blob, b.off, np.where(own == 1, hiprl.NIL_RULE, b.rule).astype(np.uint32), b.req_of,
                                b.now, b.hits))
    est, ethr = o.submit(routing.concat_batches(part))
    d0 = r0 = 0
    for g, (b, (st, thr)) in enumerate(zip(steps[10], got)):
        own = routing.owners_of(b, RULES, G, SEED)
        e_st = est[d0:d0 + b.n_desc].copy()
        e_st[own == 1] = (0, 0, 0, 0, 0)  # RL_CODE_UNKNOWN
        streams.assert_same(e_st, ethr[r0:r0 + b.n_req], st, thr, f"partial step origin={g}")
        d0 += b.n_desc
        r0 += b.n_req
    r2.close()
    r.close()

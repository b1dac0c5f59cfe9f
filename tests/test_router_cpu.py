"""Multi-GPU routing protocol on CPU: world_size-2 (and 3) gloo runs of router.ShardRouter.

Each rank is an origin with its own seeded request stream and the owner of the keys that
route_owner assigns to it. The shards are tests/routing.OracleShard (the device byte
layouts, the CPU oracle as owner), so this checks the exchange itself: count all-to-all,
variable-split record all-to-all, reverse reply all-to-all, perm / ThrottleMillis
reduction at the origin, and owner state carried across steps. The result of every step
must equal one serial oracle over the origins' batches in rank order.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
for p in (HERE, ROOT / "api-ratelimit_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import hiprl  # noqa: E402
import oracle  # noqa: E402
import routing  # noqa: E402
import streams  # noqa: E402

STEPS = 4


def rank_batches(rank, local_cache):
    """STEPS batches of one origin: its own keys plus keys shared by every origin."""
    reqs = streams.make_stream(100 + rank, 160 * STEPS, t0=1_700_000_000 + 0, keyspace=12, dt_max=1)
    out, i = [], 0
    per = len(reqs) // STEPS
    for s in range(STEPS):
        chunk = reqs[i:i + per]
        # every origin's step s shares one time so the serial order is well defined per window
        chunk = [(d, de, ru, h, 1_700_000_000 + s) for d, de, ru, h, _ in chunk]
        out.append(hiprl.build_batch(chunk))
        i += per
    return out


def _worker(rank, world, port, local_cache, outdir):
    import torch.distributed as dist

    import router

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sh = routing.OracleShard(rank, world, streams.RULES, local_cache=local_cache)
        r = router.ShardRouter(sh)
        res = {}
        for s, b in enumerate(rank_batches(rank, local_cache)):
            st, thr = r.step(b)
            res[f"st{s}"] = st
            res[f"thr{s}"] = thr
            res[f"recv{s}"] = np.array([r.last_recv])
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,local_cache", [(2, False), (2, True), (3, True)])
def test_routed_steps_equal_serial_oracle(tmp_path, world, local_cache):
    mp.spawn(_worker, args=(world, _free_port(), local_cache, str(tmp_path)), nprocs=world, join=True)
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    per_rank = [rank_batches(r, local_cache) for r in range(world)]
    o = oracle.Oracle(local_cache=local_cache)
    o.load_rules(streams.RULES)
    for s in range(STEPS):
        cat = routing.concat_batches([per_rank[r][s] for r in range(world)])
        est, ethr = o.submit(cat)
        d0 = r0 = 0
        for r in range(world):
            b = per_rank[r][s]
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], got[r][f"st{s}"], got[r][f"thr{s}"],
                                f"world={world} step={s} rank={r}")
            d0 += b.n_desc
            r0 += b.n_req
        # every routed descriptor was decided by exactly one owner
        n_routed = sum(int((per_rank[r][s].rule != hiprl.NIL_RULE).sum()) for r in range(world))
        assert sum(int(got[r][f"recv{s}"][0]) for r in range(world)) == n_routed
    assert (est["code_flags"] & 0xFF == hiprl.CODE_OVER_LIMIT).any()  # the stream does reach the limits


def test_owner_partition_is_balanced_and_window_independent():
    """route_owner depends on the prefix lanes only (every window of a key lands on one
    shard) and spreads keys evenly."""
    rng = np.random.default_rng(0)
    prefixes = [f"dom_k_{int(x)}_".encode() for x in rng.integers(0, 1 << 40, 4000)]
    for g in (2, 3, 8):
        own = np.array([oracle.route_owner(*oracle.prefix_lanes(p, 7), g) for p in prefixes])
        cnt = np.bincount(own, minlength=g)
        assert cnt.min() > 0.8 * len(prefixes) / g, cnt


class FailingShard(routing.OracleShard):
    """An OracleShard that fails to pack at (rank, step) pack_at and to decide at decide_at."""

    def __init__(self, *a, pack_at=None, decide_at=None, **kw):
        super().__init__(*a, **kw)
        self.step_no, self.pack_at, self.decide_at = 0, pack_at, decide_at

    def pack(self, b):
        self.step_no += 1
        if self.pack_at == self.step_no - 1:
            raise hiprl.RedisError("rl_route_pack: RL_EINVAL: injected bad batch", -1)
        return super().pack(b)

    def decide(self, recv, n):
        if self.decide_at == self.step_no - 1:
            raise hiprl.RedisError("rl_wait: RL_ENOSPC: injected full region", -3)
        return super().decide(recv, n)


def _fail_worker(rank, world, port, outdir):
    import torch.distributed as dist

    import router

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sh = FailingShard(rank, world, streams.RULES, local_cache=True,
                          pack_at=1 if rank == 1 else None, decide_at=3 if rank == 0 else None)
        r = router.ShardRouter(sh)
        res = {}
        for s, b in enumerate(rank_batches(rank, True)):
            try:
                st, thr = r.step(b)
                res[f"st{s}"], res[f"thr{s}"] = st, thr
                res[f"err{s}"] = np.array([0])
            except hiprl.RedisError as ex:
                res[f"err{s}"] = np.array([ex.code])
            res[f"status{s}"] = np.array(r.last_status)
        dist.barrier()  # every rank left every step: nobody is stuck in a collective
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def test_shard_errors_reach_every_rank(tmp_path):
    """Rank 1 fails to pack at step 1 and rank 0 fails to decide at step 3: every rank raises at
    both steps (the failing one its own code, the other RL_EPEER) and no collective hangs;
    steps 0 and 2 still equal the serial oracle (a pack failure changes no owner's state)."""
    world = 2
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert [int(got[r]["err1"][0]) for r in range(world)] == [-7, -1]
    assert [int(got[r]["err3"][0]) for r in range(world)] == [-3, -7]
    assert list(got[0]["status1"]) == [0, -1] and list(got[1]["status3"]) == [-3, 0]
    per_rank = [rank_batches(r, True) for r in range(world)]
    o = oracle.Oracle(local_cache=True)
    o.load_rules(streams.RULES)
    for s in (0, 2):
        est, ethr = o.submit(routing.concat_batches([per_rank[r][s] for r in range(world)]))
        d0 = r0 = 0
        for r in range(world):
            b = per_rank[r][s]
            assert int(got[r][f"err{s}"][0]) == 0
            streams.assert_same(est[d0:d0 + b.n_desc], ethr[r0:r0 + b.n_req], got[r][f"st{s}"], got[r][f"thr{s}"],
                                f"step={s} rank={r}")
            d0 += b.n_desc
            r0 += b.n_req

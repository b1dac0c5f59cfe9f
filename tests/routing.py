"""Test helpers for the multi-GPU router (api-ratelimit_amd/router.py).

- concat_batches: the serial stream a routed step is equivalent to (origin batches in
  rank order, request ids renumbered) — what the single oracle replays.
- OracleShard: a CPU shard with the product's byte layouts (32-B records, 24-B replies,
  perm / counts semantics of include/rl_hip.h) whose owner side is the CPU oracle, so the
  exchange protocol runs over gloo without a GPU. Records carry the oracle-restated prefix
  lanes (oracle.prefix_lanes) and owners (oracle.route_owner); the owner keys its oracle by
  the 16 lane bytes, which identify the prefix exactly as the device does.
- exchange_local: steps 2/3/5 of router.ShardRouter done by slicing, for G shards in one
  process (the GPU test drives G engines on one GPU through it).
TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import numpy as np
import torch

import hiprl
import oracle

REC_DTYPE = np.dtype([("a", "<u8"), ("b", "<u8"), ("now", "<u4"), ("rule", "<u4"), ("h", "<u4"), ("greq", "<u4")])
REPLY_DTYPE = np.dtype([("st", hiprl.STATUS_DTYPE), ("thr", "<u4")])
assert REC_DTYPE.itemsize == hiprl.ROUTE_RECORD_BYTES and REPLY_DTYPE.itemsize == hiprl.ROUTE_REPLY_BYTES
REQ_BITS = 27


def concat_batches(batches):
    blobs, offs, rules, reqs, nows, hits = [], [], [], [], [], []
    boff, roff = 0, 0
    for b in batches:
        blobs.append(b.blob[:int(b.off[-1])])  # (a generated blob may carry slack past its last prefix)
        offs.append(b.off[:-1].astype(np.int64) + boff)
        rules.append(b.rule)
        reqs.append(b.req_of.astype(np.int64) + roff)
        nows.append(b.now)
        hits.append(b.hits)
        boff += int(b.off[-1])
        roff += b.n_req
    off = np.concatenate(offs + [np.array([boff])]).astype(np.uint32)
    jit = None
    if any(getattr(b, "jit", None) is not None for b in batches):
        jit = np.concatenate([b.jit if b.jit is not None else np.zeros(b.n_desc, np.uint16) for b in batches])
    return hiprl.Batch(np.concatenate(blobs).astype(np.uint8), off, np.concatenate(rules).astype(np.uint32),
                       np.concatenate(reqs).astype(np.uint32), np.concatenate(nows).astype(np.int64),
                       np.concatenate(hits).astype(np.uint32), None if jit is None else jit.astype(np.uint16))


def owners_of(b, rules, n_shards, seed):
    """Owner shard of every descriptor per the oracle restatement (-1 for a nil limit)."""
    own = np.full(b.n_desc, -1, np.int64)
    for i in range(b.n_desc):
        r = int(b.rule[i])
        if r == hiprl.NIL_RULE:
            continue
        a, bb = oracle.prefix_lanes(b.prefix(i), seed)
        own[i] = oracle.route_owner(a, bb, n_shards)
    return own


class OracleShard:
    """CPU shard: pack / decide / unpack with the device's byte layouts, oracle as owner."""

    def __init__(self, rank, world, rules, seed=0x5EE7AB1E5EED, local_cache=False, ratio=0.8):
        self.rank, self.world, self.rules, self.seed = rank, world, rules, seed
        self.o = oracle.Oracle(near_limit_ratio=ratio, local_cache=local_cache)
        self.o.load_rules(rules)

    def empty(self, nbytes):
        return torch.empty(nbytes, dtype=torch.uint8)

    def pack(self, b):
        own = owners_of(b, self.rules, self.world, self.seed)
        rec = np.zeros(b.n_desc, REC_DTYPE)
        for i in range(b.n_desc):
            if own[i] < 0:
                continue
            r = int(b.rule[i])
            q = int(b.req_of[i])
            a, bb = oracle.prefix_lanes(b.prefix(i), self.seed)
            rec[i] = (a, bb, int(b.now[q]), r, max(1, int(b.hits[q])), (self.rank << REQ_BITS) | q)
        order = np.argsort(np.where(own < 0, self.world, own), kind="stable")
        counts = [int((own == s).sum()) for s in range(self.world)]
        n_routed = sum(counts)
        perm = np.full(b.n_desc, hiprl.ROUTE_LOCAL, np.uint32)
        perm[order[:n_routed]] = np.arange(n_routed, dtype=np.uint32)
        send = torch.from_numpy(rec[order[:n_routed]].view(np.uint8).copy())
        return send, torch.tensor(counts, dtype=torch.int32), counts, perm

    def decide(self, recv, n):
        rec = recv.numpy().view(REC_DTYPE)
        assert len(rec) == n
        # one owner-side request per run of equal greq (records of a request are adjacent)
        blob = np.ascontiguousarray(np.stack([rec["a"], rec["b"]], axis=1)).view(np.uint8).reshape(-1)
        new_req = np.ones(n, bool)
        new_req[1:] = rec["greq"][1:] != rec["greq"][:-1]
        req_of = (np.cumsum(new_req) - 1).astype(np.uint32)
        starts = np.flatnonzero(new_req)
        b = hiprl.Batch(blob.copy(), (np.arange(n + 1) * 16).astype(np.uint32), rec["rule"].astype(np.uint32),
                        req_of, rec["now"][starts].astype(np.int64), rec["h"][starts].astype(np.uint32))
        st, thr = self.o.submit(b) if n else (np.zeros(0, hiprl.STATUS_DTYPE), np.zeros(0, np.uint32))
        rep = np.zeros(n, REPLY_DTYPE)
        rep["st"] = st
        rep["thr"] = thr[req_of] if n else 0
        return torch.from_numpy(rep.view(np.uint8).copy())

    def unpack(self, b, perm, back):
        rep = back.numpy().view(REPLY_DTYPE)
        out = np.zeros(b.n_desc, hiprl.STATUS_DTYPE)
        thr = np.zeros(b.n_req, np.uint32)
        for i in range(b.n_desc):
            p = int(perm[i])
            if p == hiprl.ROUTE_LOCAL:
                out[i] = (hiprl.CODE_OK, 0, 0, 0, 0)
                continue
            out[i] = rep[p]["st"]
            q = int(b.req_of[i])
            thr[q] = max(thr[q], int(rep[p]["thr"]))
        return out, thr


def exchange_local(shards, batches):
    """One routed step of len(shards) shards in one process: the all-to-alls by slicing."""
    G = len(shards)
    packed = [sh.pack(b) for sh, b in zip(shards, batches)]
    offs = [np.concatenate([[0], np.cumsum(p[2])]) for p in packed]
    R, P = hiprl.ROUTE_RECORD_BYTES, hiprl.ROUTE_REPLY_BYTES
    replies = []
    for j in range(G):
        parts = [packed[i][0][offs[i][j] * R:offs[i][j + 1] * R] for i in range(G)]
        recv = torch.cat(parts) if parts else shards[j].empty(0)
        replies.append(shards[j].decide(recv, int(recv.numel() // R)))
    outs = []
    for i in range(G):
        parts = []
        for j in range(G):
            roff = sum(packed[k][2][j] for k in range(i))  # origin i's chunk inside owner j's reply
            parts.append(replies[j][roff * P:(roff + packed[i][2][j]) * P])
        back = torch.cat(parts)
        outs.append(shards[i].unpack(batches[i], packed[i][3], back))
    return outs, [p[2] for p in packed]

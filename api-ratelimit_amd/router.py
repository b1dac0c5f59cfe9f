"""Multi-GPU routed DoLimit step (include/rl_hip.h "Multi-GPU router").

One process per GPU. The key space is hash-sharded one shard per GPU: the owner of a key is
a mix of its prefix fingerprint lanes (rl_common.h route_owner), so every window of a key
and every origin agree on it — the analogue of the reference sending each key's INCRBY to
the Redis server that holds it (src/redis/fixed_cache_impl.go:66-80,
src/redis/driver_impl.go:56-90). One step of a rank:

  1. pack      its own batch -> 32-B records grouped by owner (+ counts, perm)
  2. all-to-all of the per-owner counts
  3. all-to-all of the records (variable splits)
  4. decide    the records received from every origin, origin-major (the owner's engine)
  5. all-to-all of the 24-B replies (reverse splits)
  6. unpack    replies -> rl_status[n_desc] and ThrottleMillis[n_req] in its own order

A shard whose pack or decide fails still takes part in every exchange of the step: the
counts all-to-all carries each origin's pack status next to its counts, and a status
all-to-all after the owners decide carries each owner's (the replies are exchanged and
unpacked either way). Every rank then raises together (its own error, or RL_EPEER naming
the failed shard), so one bad batch cannot leave the other GPUs blocked in a collective.
A step synchronises the host twice: once for the counts (send and receive sizes of the
record exchange), once for the owners' statuses at its end.

The exchange is plain torch.distributed (RCCL over xGMI for "nccl", gloo on CPU for the
tests); the shard object does steps 1, 4 and 6. EngineShard is the product shard (HIP
engine, device tensors); a test shard with the same byte layouts can stand in on CPU.

An owner decides what it receives as if the origins' batches had been submitted to one
engine in rank order, so the multi-GPU result equals one serial DoLimit stream.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

import hiprl

REC = hiprl.ROUTE_RECORD_BYTES
REP = hiprl.ROUTE_REPLY_BYTES
STATUS_BYTES = 20


@dataclass
class DeviceBatch:
    """A flat batch (rl_batch layout) resident on the shard's device."""
    blob: torch.Tensor   # uint8
    off: torch.Tensor    # int32 [n_desc + 1]
    rule: torch.Tensor   # int32 [n_desc]
    req_of: torch.Tensor  # int32 [n_desc]
    now: torch.Tensor    # int64 [n_req]
    hits: torch.Tensor   # int32 [n_req]
    nbytes: int = -1     # prefix bytes used (off[-1]); -1 = read it from the device
    jit: Optional[torch.Tensor] = None  # int16 [n_desc] (uint16 EXPIRE jitter) or None

    @property
    def n_desc(self) -> int:
        return int(self.rule.shape[0])

    @property
    def n_req(self) -> int:
        return int(self.now.shape[0])

    @classmethod
    def from_host(cls, b: "hiprl.Batch", device) -> "DeviceBatch":
        import numpy as np

        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        # the device reads prefix bytes as 16-B loads: the blob is readable RL_BLOB_SLACK bytes past its end
        blob = np.zeros(int(b.blob.shape[0]) + hiprl.BLOB_SLACK, np.uint8)
        blob[:b.blob.shape[0]] = b.blob
        jit = getattr(b, "jit", None)
        return cls(t(blob), t(b.off.view(np.int32)), t(b.rule.view(np.int32)), t(b.req_of.view(np.int32)),
                   t(b.now), t(b.hits.view(np.int32)), int(b.off[-1]),
                   None if jit is None else t(np.ascontiguousarray(jit, np.uint16).view(np.int16)))

    def ptrs(self):
        return [self.blob.data_ptr(), self.off.data_ptr(), self.rule.data_ptr(), self.req_of.data_ptr(),
                self.now.data_ptr(), self.hits.data_ptr(), 0 if self.jit is None else self.jit.data_ptr()]

    def blob_bytes(self) -> int:
        if self.nbytes < 0:
            self.nbytes = int(self.off[-1].item()) if self.n_desc else 0
        return self.nbytes


class EngineShard:
    """The product shard: one hiprl.Engine on this rank's GPU, on a stream of its own that is
    ordered against the caller's current stream by device-side waits in both directions around
    every call (RCCL collectives run on the caller's stream, so no host waits are needed between
    steps beyond the count exchange and the owner's batch). A dedicated stream, not the
    caller's: torch's default stream is the HIP null stream, which has no handle to pass over
    the C ABI (NULL there means the engine's own, non-blocking stream)."""

    def __init__(self, engine: "hiprl.Engine", rank: int, world: int, device, max_desc: int):
        if world > hiprl.ROUTE_MAX_SHARDS:
            raise ValueError(f"at most {hiprl.ROUTE_MAX_SHARDS} shards")
        self.eng, self.rank, self.world, self.device = engine, rank, world, device
        self.stream = torch.cuda.Stream(device)
        self.eng.set_stream(self.stream.cuda_stream)
        self.send = torch.empty(max_desc * REC, dtype=torch.uint8, device=device)
        self.perm = torch.empty(max(1, max_desc), dtype=torch.int32, device=device)
        self.counts = torch.empty(world, dtype=torch.int32, device=device)

    def empty(self, nbytes: int) -> torch.Tensor:
        return torch.empty(nbytes, dtype=torch.uint8, device=self.device)

    def _enter(self):
        self.stream.wait_stream(torch.cuda.current_stream(self.device))  # inputs written by the caller

    def _leave(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)  # outputs used by the caller

    def pack(self, b: DeviceBatch):
        self._enter()
        counts = self.eng.route_pack(b.n_desc, b.n_req, b.blob_bytes(), b.ptrs(), self.rank, self.world,
                                     self.send.data_ptr(), self.counts.data_ptr(), self.perm.data_ptr())
        self._leave()
        return self.send[:sum(counts) * REC], self.counts, counts, self.perm[:b.n_desc]

    def pack_async(self, b: DeviceBatch):
        """pack without a host round trip: the (count, status) pair for every owner lands in a
        device tensor, ready for the all-to-all of counts (ShardRouter.step)."""
        x = torch.empty(2 * self.world, dtype=torch.int32, device=self.device)
        self._enter()
        self.eng.route_pack_async(b.n_desc, b.n_req, b.blob_bytes(), b.ptrs(), self.rank, self.world,
                                  self.send.data_ptr(), x.data_ptr(), self.perm.data_ptr())
        self._leave()
        return self.send, x, self.perm[:b.n_desc]

    def decide(self, recv: torch.Tensor, n: int) -> torch.Tensor:
        reply = self.empty(n * REP)
        self._enter()
        self.eng.submit_routed_async(recv.data_ptr() if n else 0, n, reply.data_ptr() if n else 0)
        self.eng.wait()
        self._leave()
        return reply

    def unpack(self, b: DeviceBatch, perm: torch.Tensor, back: torch.Tensor):
        out = self.empty(b.n_desc * STATUS_BYTES)
        thr = torch.empty(b.n_req, dtype=torch.int32, device=self.device)
        self._enter()
        self.eng.route_unpack(b.n_desc, b.n_req, b.req_of.data_ptr(), perm.data_ptr(),
                              back.data_ptr() if back.numel() else 0, out.data_ptr(), thr.data_ptr())
        self._leave()
        return out, thr


def _code(ex: Exception) -> int:
    c = getattr(ex, "code", None)
    return int(c) if c else -1  # RL_EINVAL for errors without a C code


class ShardRouter:
    """Steps 2, 3 and 5 of the routed step over a torch.distributed group."""

    def __init__(self, shard, group=None):
        self.shard = shard
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.last_recv = 0  # records this rank decided as owner in the last step
        self.last_status = [0] * self.world  # per shard: pack / decide status of the last step

    def _raise(self, phase: str, status, own: Exception | None):
        self.last_status = status
        if own is not None:
            raise own
        bad = [j for j, c in enumerate(status) if c]
        raise hiprl.RedisError(f"routed step: RL_EPEER: shard {bad[0]} failed to {phase} "
                               f"({hiprl.RL_ERRORS.get(status[bad[0]], status[bad[0]])})", -7)

    def _pack(self, b):
        """-> (send buffer, device (count, status) pairs, perm, own error). A shard with
        pack_async packs without a host round trip: its counts come back with the all-to-all of
        counts (one host synchronisation per exchange instead of two)."""
        sh = self.shard
        if hasattr(sh, "pack_async"):
            try:
                send, x, perm = sh.pack_async(b)
                return send, x, perm, None
            except hiprl.RedisError as ex:
                own = ex
        else:
            try:
                send, _, counts, perm = sh.pack(b)
                x = torch.tensor([v for c in counts for v in (c, 0)], dtype=torch.int32, device=send.device)
                return send, x, perm, None
            except hiprl.RedisError as ex:
                own = ex
        send = sh.empty(0)
        x = torch.tensor([v for _ in range(self.world) for v in (0, _code(own))], dtype=torch.int32,
                         device=send.device)
        return send, x, None, own

    def step(self, b):
        sh = self.shard
        send, x, perm, own = self._pack(b)
        rx = torch.empty_like(x)
        dist.all_to_all_single(rx, x, group=self.group)
        both = [int(v) for v in torch.cat([x, rx]).tolist()]  # the step's one sync before the records
        counts = both[0:2 * self.world:2]
        rcounts, status = both[2 * self.world::2], both[2 * self.world + 1::2]
        if own is None and both[1]:  # the device found this batch malformed (rl_route_pack's checks)
            own = hiprl.RedisError("rl_route_pack_async: RL_EINVAL: batch references an unknown rule id or request "
                                   "index, malformed prefix offsets, or a time outside [0, 0xFFFD0000]", both[1])
        if any(status):
            self._raise("pack its batch", status, own)
        send = send[:sum(counts) * REC]
        n_in = sum(rcounts)
        recv = sh.empty(n_in * REC)
        dist.all_to_all_single(recv, send, [c * REC for c in rcounts], [c * REC for c in counts], group=self.group)
        try:
            reply = sh.decide(recv, n_in)
        except hiprl.RedisError as ex:
            own, reply = ex, sh.empty(n_in * REP)
        # The owners' statuses, the replies and the unpack are all enqueued before the host
        # waits once, at the end: a failed owner still sends (meaningless) replies of the agreed
        # sizes, and every rank raises after the exchanges, so no rank is left in a collective.
        e = torch.full((self.world,), _code(own) if own is not None else 0, dtype=torch.int32, device=x.device)
        re_ = torch.empty_like(e)
        dist.all_to_all_single(re_, e, group=self.group)
        back = sh.empty(sum(counts) * REP)
        dist.all_to_all_single(back, reply, [c * REP for c in counts], [c * REP for c in rcounts], group=self.group)
        out = sh.unpack(b, perm, back)
        status = [int(v) for v in re_.tolist()]
        if any(status):
            self._raise("decide its records", status, own)
        self.last_recv = n_in
        self.last_status = [0] * self.world
        return out

"""RESP replay of a decided batch.

The reference's Redis backend sends, per descriptor that has a limit and is not a local-cache
hit, `INCRBY key hitsAddend` then `EXPIRE key ttl` (`src/redis/fixed_cache_impl.go:26-29`,
skips at `:57-66`), each encoded by radix v3.5.1 `FlatCmd` (`src/redis/driver_impl.go:138,150`)
as a RESP array of bulk strings with integers in decimal. SECOND keys go to the per-second
client when `REDIS_PERSECOND` is set (`fixed_cache_impl.go:74-85`).

This module rebuilds that exact byte stream from a batch and the statuses the HIP engine (or
the oracle) returned for it, so the decisions can be checked against a live redis-server:
replay the stream, read the INCRBY replies, and `check_replies` asserts that every status is
the one `GetResponseDescriptorStatus` gives for that post-value (`src/limiter/base_limiter.go:
70-115`, thresholds `:129-177`). No redis-server exists in this image or on the GPU box, so the
tests replay into `RespStore`, a minimal in-process RESP executor with Redis' INCRBY/EXPIRE
semantics (missing key = 0, post-increment reply); the live path (`replay_to_redis`) runs only
when `RL_REDIS_ADDR` names a server. Expiry is not simulated: keys carry their window start
(`src/limiter/cache_key.go:57-68`), so a window never reuses an earlier window's key.
"""
from __future__ import annotations

import socket
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

import hiprl

CRLF = b"\r\n"


def _bulk(x) -> bytes:
    if isinstance(x, bytes):
        b = x
    elif isinstance(x, str):
        b = x.encode()
    elif isinstance(x, (int, np.integer)):
        b = str(int(x)).encode()  # radix FlatCmd writes integers in decimal
    else:
        raise TypeError(f"unsupported RESP argument {type(x)}")
    return b"$" + str(len(b)).encode() + CRLF + b + CRLF


def flat_cmd(cmd: str, key, *args) -> bytes:
    """radix.FlatCmd(rcv, cmd, key, args...) on the wire: `*N` then N bulk strings."""
    parts = [cmd, key, *args]
    return b"*" + str(len(parts)).encode() + CRLF + b"".join(_bulk(p) for p in parts)


def cache_key(prefix: bytes, unit: int, now: int) -> bytes:
    """prefix || decimal((now / div) * div)  (cache_key.go:57-68, utilities.go:19-32)."""
    div = hiprl.UNIT_DIVIDER[unit]
    return prefix + str((int(now) // div) * div).encode()


class Command:
    __slots__ = ("desc", "key", "hits", "ttl", "per_second")

    def __init__(self, desc, key, hits, ttl, per_second):
        self.desc, self.key, self.hits, self.ttl, self.per_second = desc, key, hits, ttl, per_second


def commands(batch: hiprl.Batch, rules: Sequence[Tuple[int, int]], status: np.ndarray,
             per_second_split: bool = False, jitter: Optional[Callable[[], int]] = None) -> List[Command]:
    """The INCRBY/EXPIRE pairs of a batch in serial order (fixed_cache_impl.go:55-86).

    rules[i] = (requests_per_unit, unit); status = the engine's rl_status array for the batch
    (its LOCAL_CACHE_HIT flag marks the descriptors the reference skips, `:61-66`). jitter()
    returns `JitterRand.Int63n(ExpirationJitterMaxSeconds)` (`:69-72`), 0 when None."""
    out = []
    for i in range(batch.n_desc):
        rid = int(batch.rule[i])
        if rid == hiprl.NIL_RULE:
            continue  # cacheKey.Key == "" (`:57-59`)
        if (int(status[i]["code_flags"]) >> 8) & hiprl.FLAG_LOCAL_CACHE_HIT:
            continue
        unit = rules[rid][1]
        r = int(batch.req_of[i])
        h = max(1, int(batch.hits[r]))  # utils.Max(1, request.HitsAddend) (`:39`)
        ttl = hiprl.UNIT_DIVIDER[unit] + (int(jitter()) if jitter else 0)
        out.append(Command(i, cache_key(batch.prefix(i), unit, int(batch.now[r])), h, ttl,
                           per_second_split and unit == hiprl.SECOND))
    return out


def encode(cmds: Sequence[Command]) -> Tuple[bytes, bytes]:
    """(main client stream, per-second client stream)."""
    main, ps = bytearray(), bytearray()
    for c in cmds:
        dst = ps if c.per_second else main
        dst += flat_cmd("INCRBY", c.key, c.hits)
        dst += flat_cmd("EXPIRE", c.key, c.ttl)
    return bytes(main), bytes(ps)


def parse_replies(data: bytes) -> List[int]:
    """Integer replies of a pipelined stream; an error reply raises hiprl.RedisError, the
    backend's failure convention (src/redis/driver.go:6-10)."""
    out, i = [], 0
    while i < len(data):
        j = data.index(CRLF, i)
        t, body = data[i:i + 1], data[i + 1:j]
        if t == b":":
            out.append(int(body))
        elif t == b"-":
            raise hiprl.RedisError(body.decode(errors="replace"))
        else:
            raise hiprl.RedisError(f"unexpected RESP reply type {t!r}")
        i = j + 2
    return out


def _parse_commands(data: bytes):
    i = 0
    while i < len(data):
        if data[i:i + 1] != b"*":
            raise ValueError("RESP command must be an array")
        j = data.index(CRLF, i)
        n = int(data[i + 1:j])
        i = j + 2
        parts = []
        for _ in range(n):
            j = data.index(CRLF, i)
            ln = int(data[i + 1:j])
            parts.append(data[j + 2:j + 2 + ln])
            i = j + 2 + ln + 2
        yield parts


class RespStore:
    """A minimal RESP executor for INCRBY/EXPIRE with Redis' semantics: INCRBY on a missing
    key starts from 0 and replies the post-value; EXPIRE replies 1 if the key exists."""

    def __init__(self):
        self.counters: Dict[bytes, int] = {}
        self.ttl: Dict[bytes, int] = {}

    def execute(self, data: bytes) -> bytes:
        out = bytearray()
        for parts in _parse_commands(data):
            cmd = parts[0].upper()
            if cmd == b"INCRBY":
                v = self.counters.get(parts[1], 0) + int(parts[2])
                self.counters[parts[1]] = v
                out += b":" + str(v).encode() + CRLF
            elif cmd == b"EXPIRE":
                ok = parts[1] in self.counters
                if ok:
                    self.ttl[parts[1]] = int(parts[2])
                out += b":1\r\n" if ok else b":0\r\n"
            else:
                out += b"-ERR unknown command '" + parts[0] + b"'\r\n"
        return bytes(out)


def replay_to_redis(data: bytes, host: str, port: int, n_replies: int, timeout: float = 10.0) -> bytes:
    """Send a pipelined stream to a live redis-server and read exactly n_replies replies."""
    with socket.create_connection((host, port), timeout=timeout) as s:
        s.sendall(data)
        buf = bytearray()
        while buf.count(CRLF) < n_replies:
            chunk = s.recv(1 << 16)
            if not chunk:
                raise hiprl.RedisError("connection closed by redis-server")
            buf += chunk
        return bytes(buf)


def check_replies(batch: hiprl.Batch, rules: Sequence[Tuple[int, int]], status: np.ndarray,
                  cmds: Sequence[Command], incr: Sequence[int]) -> None:
    """Assert each status is what GetResponseDescriptorStatus gives for its INCRBY reply
    `after` (base_limiter.go:83-113, 129-145): OK ⇔ after ≤ L with remaining = L − after;
    OVER_LIMIT ⇔ after > L with Δover = after − L, or h when before = after − h ≥ L."""
    assert len(cmds) == len(incr)
    for c, after in zip(cmds, incr):
        L = rules[int(batch.rule[c.desc])][0]
        s = status[c.desc]
        code = int(s["code_flags"]) & 0xFF
        after32 = after & 0xFFFFFFFF  # results[i] is a uint32 (fixed_cache_impl.go:51)
        if after32 > L:
            assert code == hiprl.CODE_OVER_LIMIT, (c.key, after, L, code)
            assert int(s["limit_remaining"]) == 0, (c.key, after)
            dov = int(s["over_limit_delta"])
            before = (after32 - c.hits) & 0xFFFFFFFF
            assert dov == (c.hits if before >= L else after32 - L), (c.key, after, L, dov)
        else:
            assert code == hiprl.CODE_OK, (c.key, after, L, code)
            assert int(s["limit_remaining"]) == L - after32, (c.key, after, L, int(s["limit_remaining"]))


def incr_replies(cmds: Sequence[Command], main_replies: Sequence[int], ps_replies: Sequence[int]) -> List[int]:
    """INCRBY post-value of every command, from the two clients' reply lists (each stream
    replies INCRBY, EXPIRE, INCRBY, EXPIRE, ... in its own order)."""
    it = {False: iter(main_replies[0::2]), True: iter(ps_replies[0::2])}
    return [next(it[c.per_second]) for c in cmds]


def replay_local(store: RespStore, ps_store: Optional[RespStore], batch: hiprl.Batch,
                 rules: Sequence[Tuple[int, int]], status: np.ndarray, per_second_split: bool = False) -> List[int]:
    """Encode a decided batch, execute it on the stand-in store(s), check every status against
    its INCRBY reply, and return the replies."""
    cmds = commands(batch, rules, status, per_second_split)
    main, ps = encode(cmds)
    r_main = parse_replies(store.execute(main))
    r_ps = parse_replies((ps_store if ps_store is not None else store).execute(ps)) if ps else []
    incr = incr_replies(cmds, r_main, r_ps)
    check_replies(batch, rules, status, cmds, incr)
    return incr

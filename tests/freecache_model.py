"""Test infrastructure: a pure-Python restatement of coocood/freecache v1.1.0's eviction (the
reference's local over-limit cache, go.mod:9; created at src/service_cmd/runner/runner.go:85-88,
used at src/limiter/base_limiter.go:57-66,94-106), written independently of the product's C++
model (api-ratelimit_amd/csrc/rl_freecache.hpp) so the two can be checked against each other.

PARITY UNPINNED: freecache is not in this image and the reference's tests hold no vector that
exercises its eviction (base_limiter_test.go uses a 100-byte cache, raised to freecache's
512-KiB floor, without filling it). Time is the caller's (request) time in seconds.
"""
from __future__ import annotations

from collections import OrderedDict

import xxhash

SEGMENTS = 256
MIN_BYTES = 512 * 1024
ENTRY_HDR = 24


def segment_of(key: bytes) -> int:
    return xxhash.xxh64_intdigest(key) & (SEGMENTS - 1)  # hashVal & segmentAndOpVal


class _Entry:
    __slots__ = ("key", "access", "expire", "length", "deleted")

    def __init__(self, key, access, expire, length):
        self.key, self.access, self.expire, self.length, self.deleted = key, access, expire, length, False


class _Segment:
    def __init__(self, cap: int):
        self.cap = cap
        self.vacuum = cap
        self.ring: "OrderedDict[int, _Entry]" = OrderedDict()  # ring order, oldest first
        self.index: dict[bytes, int] = {}
        self.total_count = 0
        self.total_time = 0
        self._next = 0

    def append(self, e: _Entry) -> int:
        self._next += 1
        self.ring[self._next] = e
        return self._next


class FreeCache:
    def __init__(self, size: int):
        size = max(size, MIN_BYTES)
        self.segs = [_Segment(size // SEGMENTS) for _ in range(SEGMENTS)]
        self.hits = self.misses = self.lookups = self.evacuated = self.expired = 0

    def get(self, key: bytes, now: int) -> bool:
        s = self.segs[segment_of(key)]
        self.lookups += 1
        h = s.index.get(key)
        if h is None:
            self.misses += 1
            return False
        e = s.ring[h]
        if e.expire != 0 and e.expire <= now:
            e.deleted = True
            del s.index[key]
            self.expired += 1
            self.misses += 1
            return False
        s.total_time += (now - e.access) & 0xFFFFFFFF  # int64(uint32(now - accessTime))
        e.access = now
        self.hits += 1
        return True

    def set(self, key: bytes, ttl: int, now: int) -> bool:
        s = self.segs[segment_of(key)]
        if len(key) > 65535 or len(key) + ENTRY_HDR > s.cap // 4:
            return False
        expire = (now + ttl) & 0xFFFFFFFF if ttl > 0 else 0
        h = s.index.get(key)
        if h is not None:  # in place: the empty value fits the entry's 1-byte capacity
            e = s.ring[h]
            s.total_time += now - e.access
            e.access, e.expire = now, expire
            return True
        length = ENTRY_HDR + len(key) + 1
        self._evacuate(s, length, now)
        s.index[key] = s.append(_Entry(key, now, expire, length))
        s.total_time += now
        s.total_count += 1
        s.vacuum -= length
        return True

    def _evacuate(self, s: _Segment, length: int, now: int):
        moves = 0
        while s.vacuum < length:
            h, e = next(iter(s.ring.items()))
            if e.deleted:
                moves = 0
                s.total_time -= e.access
                s.total_count -= 1
                s.vacuum += e.length
                del s.ring[h]
                continue
            expired = e.expire != 0 and e.expire < now
            if expired or e.access * s.total_count <= s.total_time or moves > 5:
                moves = 0
                s.total_time -= e.access
                s.total_count -= 1
                s.vacuum += e.length
                if expired:
                    self.expired += 1
                else:
                    self.evacuated += 1
                del s.index[e.key]
                del s.ring[h]
            else:  # recently used: to the ring's newest end
                del s.ring[h]
                s.index[e.key] = s.append(e)
                moves += 1

    def entries(self) -> int:
        return sum(len(s.index) for s in self.segs)

    def stats(self):
        return [self.hits, self.misses, self.lookups, self.entries(), self.evacuated, self.expired]

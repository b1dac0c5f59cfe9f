"""ctypes harness of the CPU oracle (oracle/rl_oracle.cpp) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this,
and only as the checker / CPU baseline. The product path (api-ratelimit_amd/) never
imports it. Parity pinning of the oracle itself: tests/test_oracle_golden.py against
the vectors in tests/golden/reference_vectors.json (transcribed from the reference's
test/redis/fixed_cache_impl_test.go, test/limiter/base_limiter_test.go and
test/integration/integration_test.go).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "librl_oracle.so"

STATUS_DTYPE = np.dtype([("code_flags", "<u4"), ("limit_remaining", "<u4"), ("reset_s", "<u4"),
                         ("over_limit_delta", "<u4"), ("near_limit_delta", "<u4")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        vp, u32, i64, u64 = C.c_void_p, C.c_uint32, C.c_int64, C.c_uint64
        L.rlo_create.argtypes = [C.c_float, C.c_int, C.c_int]
        L.rlo_create.restype = vp
        L.rlo_destroy.argtypes = [vp]
        L.rlo_load_rules.argtypes = [vp, vp, u32]
        L.rlo_load_rules.restype = C.c_int
        sub = [vp, u32, vp, vp, vp, vp, u32, vp, vp, vp, vp, vp]
        L.rlo_submit.argtypes = sub
        L.rlo_submit.restype = C.c_int
        L.rlo_submit_mt.argtypes = [vp, C.c_int] + sub[1:]
        L.rlo_submit_mt.restype = C.c_int
        L.rlo_decide.argtypes = [u32, u32, C.c_float, i64, u32, u32, u32, C.c_int, C.c_int, vp, vp]
        L.rlo_decide.restype = None
        L.rlo_cache_key.argtypes = [C.c_char_p, u32, u32, i64, C.c_char_p, u32]
        L.rlo_cache_key.restype = u32
        L.rlo_counter.argtypes = [vp, C.c_char_p, u32, C.c_int, i64]
        L.rlo_counter.restype = i64
        L.rlo_local_cached.argtypes = [vp, C.c_char_p, u32, i64]
        L.rlo_local_cached.restype = C.c_int
        L.rlo_num_keys.argtypes = [vp]
        L.rlo_num_keys.restype = u64
        L.rlo_num_strings.argtypes = [vp]
        L.rlo_num_strings.restype = u64
        L.rlo_fingerprint.argtypes = [C.c_char_p, u32, u64, u64, C.POINTER(u64), C.POINTER(u64)]
        L.rlo_fingerprint.restype = None
        L.rlo_fingerprint_many.argtypes = [vp, vp, u32, u64, u64, vp, vp]
        L.rlo_fingerprint_many.restype = None
        L.rlo_place.argtypes = [u32, C.POINTER(u32), C.POINTER(u32)]
        L.rlo_place.restype = None
        L.rlo_prefix_lanes.argtypes = [C.c_char_p, u32, u64, C.POINTER(u64), C.POINTER(u64)]
        L.rlo_prefix_lanes.restype = None
        L.rlo_route_owner.argtypes = [u64, u64, u32]
        L.rlo_route_owner.restype = u32
        L.rlo_local_cache_stats.argtypes = [vp] + [C.POINTER(u64)] * 4
        L.rlo_local_cache_stats.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a.size else None


class Oracle:
    """Serial DoLimit over a Redis stand-in; same flat batch layout as the C ABI."""

    def __init__(self, near_limit_ratio=0.8, local_cache=False, per_second_split=False):
        self.L = lib()
        self.h = self.L.rlo_create(near_limit_ratio, int(local_cache), int(per_second_split))
        self.near_limit_ratio = near_limit_ratio

    def __del__(self):
        try:
            self.L.rlo_destroy(self.h)
        except Exception:
            pass

    def load_rules(self, rules):
        # (L, unit) or (L, unit, shadow_mode): shadow rides in the unit's RLO_RULE_SHADOW bit
        arr = np.array([(r[0], r[1] | (0x100 if len(r) > 2 and r[2] else 0)) for r in rules],
                       dtype=np.uint32).reshape(-1, 2)
        rc = self.L.rlo_load_rules(self.h, _p(arr), len(rules))
        if rc:
            raise ValueError(f"rlo_load_rules: {rc}")

    def submit(self, b, threads: int = 1):
        out = np.zeros(b.n_desc, STATUS_DTYPE)
        thr = np.zeros(b.n_req, np.uint32)
        jit = getattr(b, "jit", None)  # EXPIRE jitter per descriptor (uint16), or None
        if jit is not None:
            jit = np.ascontiguousarray(jit, np.uint16)
        args = (b.n_desc, _p(b.blob), _p(b.off), _p(b.rule), _p(b.req_of), b.n_req, _p(b.now), _p(b.hits),
                None if jit is None else _p(jit), _p(out), _p(thr))
        if threads > 1:
            rc = self.L.rlo_submit_mt(self.h, threads, *args)
        else:
            rc = self.L.rlo_submit(self.h, *args)
        if rc:
            raise ValueError(f"rlo_submit: {rc}")
        return out, thr

    def counter(self, key: bytes, now=None, per_second=False) -> int:
        """Redis counter of a full key string at time `now` (-1: absent or expired); now=None
        ignores expiry (the last value INCRBY left)."""
        return self.L.rlo_counter(self.h, key, len(key), int(per_second), -(1 << 63) if now is None else now)

    def local_cached(self, key: bytes, now: int) -> bool:
        return bool(self.L.rlo_local_cached(self.h, key, len(key), now))

    def num_keys(self) -> int:
        return self.L.rlo_num_keys(self.h)

    def num_strings(self) -> int:
        """Distinct key strings ever stored (one device table slot each per window)."""
        return self.L.rlo_num_strings(self.h)

    def local_cache_stats(self) -> dict:
        v = [C.c_uint64() for _ in range(4)]
        self.L.rlo_local_cache_stats(self.h, *[C.byref(x) for x in v])
        return dict(zip(["hit", "miss", "lookup", "entries"], [x.value for x in v]))


def decide(L_, unit, ratio, now, hits, after, local_hit=False, has_limit=True, before=None):
    """GetResponseDescriptorStatus for one descriptor; before defaults to after - hits (DoLimit)."""
    out = np.zeros(1, STATUS_DTYPE)
    thr = np.zeros(1, np.uint32)
    if before is None:
        before = (after - hits) & 0xFFFFFFFF
    lib().rlo_decide(L_, unit, ratio, now, hits, before, after, int(local_hit), int(has_limit), _p(out), _p(thr))
    return out[0], int(thr[0])


def cache_key(prefix: bytes, unit: int, now: int) -> bytes:
    buf = C.create_string_buffer(len(prefix) + 32)
    n = lib().rlo_cache_key(prefix, len(prefix), unit, now, buf, len(buf))
    return buf.raw[:n]


def fingerprints(blob: np.ndarray, off: np.ndarray, window_start: int, seed: int):
    """Fingerprints (hi uint64, lo = 32-bit tag) of every key string blob[off[i]:off[i+1]] || window_start."""
    n = len(off) - 1
    hi = np.zeros(n, np.uint64)
    lo = np.zeros(n, np.uint64)
    blob = np.ascontiguousarray(blob, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    lib().rlo_fingerprint_many(_p(blob), _p(off), n, window_start, seed, _p(hi), _p(lo))
    return hi, lo


def place(window_start: int):
    """Table region (home unit x parity) and generation of a key string's window start."""
    r, g = C.c_uint32(), C.c_uint32()
    lib().rlo_place(window_start, C.byref(r), C.byref(g))
    return r.value, g.value


def prefix_lanes(prefix: bytes, seed: int):
    """Fingerprint lanes (a, b) of a key prefix before the window: the routed key identity."""
    a, b = C.c_uint64(), C.c_uint64()
    lib().rlo_prefix_lanes(prefix, len(prefix), seed, C.byref(a), C.byref(b))
    return a.value, b.value


def route_owner(a: int, b: int, n_shards: int) -> int:
    return int(lib().rlo_route_owner(a, b, n_shards))


def fingerprint(prefix: bytes, window_start: int, seed: int):
    hi, lo = C.c_uint64(), C.c_uint64()
    lib().rlo_fingerprint(prefix, len(prefix), window_start, seed, C.byref(hi), C.byref(lo))
    return hi.value, lo.value

"""Python binding of the HIP rate-limit backend (include/rl_hip.h) and a Python mirror of
the reference's backend interface, used by the parity tests and bench.py.

The product is the C ABI in libratelimit_hip.so (HIP kernels + C++ host runtime); this
module is a thin ctypes layer over it. It never falls back to a CPU implementation: if
the shared library is missing, importing `Engine` raises.

Reference interface mirrored here (for tests that read like the reference's own):
  limiter.RateLimitCache.DoLimit / Flush     src/limiter/cache.go:15-33
  limiter.DoLimitResponse                    src/limiter/cache.go:9-12
  config.RateLimit / NewRateLimit            src/config/config.go:26-32, config_impl.go:79-89
  redis.RedisError                           src/redis/driver.go:6-10
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "csrc" / "libratelimit_hip.so"

NIL_RULE = 0xFFFFFFFF
UNIT_UNKNOWN, SECOND, MINUTE, HOUR, DAY = 0, 1, 2, 3, 4
UNIT_NAMES = {SECOND: "SECOND", MINUTE: "MINUTE", HOUR: "HOUR", DAY: "DAY"}
UNIT_DIVIDER = {SECOND: 1, MINUTE: 60, HOUR: 3600, DAY: 86400}
CODE_UNKNOWN, CODE_OK, CODE_OVER_LIMIT = 0, 1, 2
FLAG_HAS_LIMIT, FLAG_LOCAL_CACHE_HIT, FLAG_SHADOW = 1, 2, 4
RULE_SHADOW = 0x100  # RL_RULE_SHADOW: shadow-mode rule (extension; rl_hip.h)

RL_ERRORS = {-1: "RL_EINVAL", -2: "RL_EHIP", -3: "RL_ENOSPC", -4: "RL_ECAPACITY", -5: "RL_ESTATE", -6: "RL_EDEVICE",
             -7: "RL_EPEER", -8: "RL_ECOMM", -9: "RL_ELATE"}

STATUS_DTYPE = np.dtype([("code_flags", "<u4"), ("limit_remaining", "<u4"), ("reset_s", "<u4"),
                         ("over_limit_delta", "<u4"), ("near_limit_delta", "<u4")])


PIPELINE_FLAGS = {"v4": 0, "lsd": 1}  # rl_config.flags (RL_CFG_LSD_ONLY)
CFG_LAG_WINDOW = 2  # RL_CFG_LAG_WINDOW: SECOND key strings findable 3 s behind (routers' engines)
ABI_VERSION = 7


class RlConfig(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("device", C.c_int32), ("log2_slots", C.c_uint32 * 4),
                ("near_limit_ratio", C.c_float), ("local_cache", C.c_uint32), ("per_second_split", C.c_uint32),
                ("max_batch_desc", C.c_uint32), ("max_batch_req", C.c_uint32), ("max_blob_bytes", C.c_uint32),
                ("sort_bits", C.c_uint32), ("flags", C.c_uint32), ("hash_seed", C.c_uint64),
                ("max_load_permille", C.c_uint32), ("reserved", C.c_uint32)]


class RlRule(C.Structure):
    _fields_ = [("requests_per_unit", C.c_uint32), ("unit", C.c_uint32)]


class RlBatch(C.Structure):
    _fields_ = [("n_desc", C.c_uint32), ("n_req", C.c_uint32), ("blob_bytes", C.c_uint32), ("reserved", C.c_uint32),
                ("prefix_blob", C.c_void_p), ("prefix_off", C.c_void_p), ("rule_id", C.c_void_p),
                ("req_of", C.c_void_p), ("now", C.c_void_p), ("hits_addend", C.c_void_p),
                ("ttl_jitter", C.c_void_p)]


class RlTreeNode(C.Structure):
    _fields_ = [("parent", C.c_uint32), ("name_off", C.c_uint32), ("name_len", C.c_uint32), ("rule", C.c_uint32)]


class RlResolveBatch(C.Structure):
    _fields_ = [("n_desc", C.c_uint32), ("n_entries", C.c_uint32), ("bytes_len", C.c_uint32), ("reserved", C.c_uint32),
                ("bytes", C.c_void_p), ("domain", C.c_void_p), ("entry_first", C.c_void_p), ("entry", C.c_void_p),
                ("override_rule", C.c_void_p)]


TREE_ROOT = 0xFFFFFFFF
BLOB_SLACK = 32  # RL_BLOB_SLACK: a device prefix_blob is readable this many bytes past its end
MAX_IN_FLIGHT = 3  # RL_MAX_IN_FLIGHT: batches in flight at once through rl_submit_pipelined


class RlEngineStats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("descriptors", C.c_uint64), ("resorts", C.c_uint64),
                ("inserted_keys", C.c_uint64), ("lsd_fallbacks", C.c_uint64), ("hot_keys", C.c_uint64),
                ("live_keys", C.c_uint64), ("host_batches", C.c_uint64)]


class RlOccupancy(C.Structure):
    _fields_ = [("gen", C.c_uint32 * 8), ("live", C.c_uint32 * 8), ("limit", C.c_uint32 * 8), ("slots", C.c_uint32 * 8)]


class RlHostBatch(C.Structure):
    _fields_ = [("prefix_blob", C.c_void_p), ("prefix_off", C.c_void_p), ("rule_id", C.c_void_p),
                ("req_of", C.c_void_p), ("now", C.c_void_p), ("hits_addend", C.c_void_p), ("ttl_jitter", C.c_void_p),
                ("max_desc", C.c_uint32), ("max_req", C.c_uint32), ("max_blob", C.c_uint32), ("reserved", C.c_uint32)]


class RlBatchC(C.Structure):
    """rl_batch_c: the compact host wire format (rl_hip.h)."""
    _fields_ = [("n_desc", C.c_uint32), ("n_req", C.c_uint32), ("blob_bytes", C.c_uint32), ("flags", C.c_uint32),
                ("now_base", C.c_int64), ("prefix_blob", C.c_void_p), ("desc_word", C.c_void_p),
                ("req_word", C.c_void_p), ("req_of", C.c_void_p), ("ttl_jitter", C.c_void_p)]


class RlHostBatchC(C.Structure):
    _fields_ = [("prefix_blob", C.c_void_p), ("desc_word", C.c_void_p), ("req_word", C.c_void_p),
                ("req_of", C.c_void_p), ("ttl_jitter", C.c_void_p), ("max_desc", C.c_uint32), ("max_req", C.c_uint32),
                ("max_blob", C.c_uint32), ("reserved", C.c_uint32)]


BC_ONE_PER_REQ = 1   # RL_BC_ONE_PER_REQ
NIL_RULE16 = 0xFFFF  # RL_NIL_RULE16
RAW_LOCAL_HIT, RAW_NIL = 1, 2  # rl_raw_reply.flags
RAW_DTYPE = np.dtype([("after", "<u4"), ("flags", "<u4")])


# (name, argtypes, restype) of every symbol include/rl_hip.h declares
class RlRouterConfig(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("n_shards", C.c_uint32), ("rank", C.c_uint32), ("max_desc", C.c_uint32),
                ("rccl_id", C.c_void_p), ("flags", C.c_uint32), ("max_blob_bytes", C.c_uint32)]


ROUTER_NO_COMBINE, ROUTER_HOST, ROUTER_EMULATED, ROUTER_HOST_XCHG = 1, 2, 4, 8  # rl_router_config.flags
# rl_host_xchg_fn: (ctx, send, send_counts, send_displs, recv, recv_counts, recv_displs) -> 0 | error
HOST_XCHG_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.c_void_p,
                           C.POINTER(C.c_size_t), C.POINTER(C.c_size_t))


class RlRouterStats(C.Structure):
    _fields_ = [("steps", C.c_uint64), ("n_shards", C.c_uint32), ("status", C.c_int32 * 16), ("recv", C.c_uint32 * 16),
                ("sent", C.c_uint32 * 16), ("pack_us", C.c_double), ("exchange_us", C.c_double),
                ("decide_us", C.c_double), ("decide_max_us", C.c_double), ("reply_us", C.c_double),
                ("unpack_us", C.c_double), ("step_us", C.c_double), ("hot_groups", C.c_uint32), ("combined", C.c_uint32),
                ("repacks", C.c_uint64), ("combined_steps", C.c_uint64), ("owner_batches", C.c_uint32),
                ("step_clock", C.c_uint32), ("late_steps", C.c_uint64)]


ROUTER_ID_BYTES = 128

ABI = [
    ("rl_create", [C.POINTER(RlConfig), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_destroy", [C.c_void_p], None),
    ("rl_last_error", [C.c_void_p], C.c_char_p),
    ("rl_abi_version", [], C.c_uint32),
    ("rl_load_rules", [C.c_void_p, C.POINTER(RlRule), C.c_uint32], C.c_int),
    ("rl_host_acquire", [C.c_void_p, C.POINTER(RlHostBatch)], C.c_int),
    ("rl_submit", [C.c_void_p, C.POINTER(RlBatch), C.c_void_p, C.c_void_p], C.c_int),
    ("rl_wait", [C.c_void_p], C.c_int),
    ("rl_query", [C.c_void_p], C.c_int),
    ("rl_wait_into", [C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("rl_wait_view", [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_host_acquire_c", [C.c_void_p, C.POINTER(RlHostBatchC)], C.c_int),
    ("rl_submit_c", [C.c_void_p, C.POINTER(RlBatchC)], C.c_int),
    ("rl_wait_raw_view", [C.c_void_p, C.POINTER(C.c_void_p)], C.c_int),
    ("rl_wait_raw_into", [C.c_void_p, C.c_void_p], C.c_int),
    ("rl_decide_raw", [C.c_void_p, C.POINTER(RlBatchC), C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p],
     C.c_int),
    ("rl_submit_device", [C.c_void_p, C.POINTER(RlBatch), C.c_void_p, C.c_void_p], C.c_int),
    ("rl_submit_pipelined", [C.c_void_p, C.POINTER(RlBatch), C.c_void_p, C.c_void_p], C.c_int),
    ("rl_stream", [C.c_void_p], C.c_void_p),
    ("rl_reset", [C.c_void_p], C.c_int),
    ("rl_get_stats", [C.c_void_p, C.POINTER(RlEngineStats)], C.c_int),
    ("rl_get_occupancy", [C.c_void_p, C.POINTER(RlOccupancy)], C.c_int),
    ("rl_set_timing", [C.c_void_p, C.c_int], C.c_int),
    ("rl_kernel_times", [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                         C.c_uint32, C.POINTER(C.c_uint32)], C.c_int),
    ("rl_last_batch_info", [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                            C.POINTER(C.c_uint64)], C.c_int),
    ("rl_set_stream", [C.c_void_p, C.c_void_p], C.c_int),
    ("rl_route_pack", [C.c_void_p, C.POINTER(RlBatch), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                       C.POINTER(C.c_uint32)], C.c_int),
    ("rl_route_pack_async", [C.c_void_p, C.POINTER(RlBatch), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                             C.c_void_p], C.c_int),
    ("rl_route_pack_strided", [C.c_void_p, C.POINTER(RlBatch), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                               C.c_void_p, C.c_void_p], C.c_int),
    ("rl_submit_routed", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p], C.c_int),
    ("rl_submit_routed_async", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p], C.c_int),
    ("rl_route_unpack", [C.c_void_p, C.POINTER(RlBatch), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    ("rl_load_tree", [C.c_void_p, C.POINTER(RlTreeNode), C.c_uint32, C.c_void_p, C.c_uint32], C.c_int),
    ("rl_resolve", [C.c_void_p, C.POINTER(RlResolveBatch), C.c_void_p], C.c_int),
    ("rl_resolve_device", [C.c_void_p, C.POINTER(RlResolveBatch), C.c_void_p], C.c_int),
    ("rl_router_unique_id", [C.c_void_p], C.c_int),
    ("rl_router_emu_world", [C.c_uint32, C.c_void_p], C.c_int),
    ("rl_router_use_host_xchg", [C.c_void_p, C.c_void_p], C.c_int),
    ("rl_router_create", [C.POINTER(RlRouterConfig), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_router_step", [C.c_void_p, C.POINTER(RlBatch), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_router_submit", [C.c_void_p, C.POINTER(RlBatch), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_router_wait", [C.c_void_p], C.c_int),
    ("rl_router_host_acquire", [C.c_void_p, C.c_uint32, C.POINTER(RlHostBatch)], C.c_int),
    ("rl_router_submit_host", [C.c_void_p, C.POINTER(RlBatch)], C.c_int),
    ("rl_router_wait_into", [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], C.c_int),
    ("rl_router_allgather_host", [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p], C.c_int),
    ("rl_router_get_stats", [C.c_void_p, C.POINTER(RlRouterStats)], C.c_int),
    ("rl_router_last_error", [C.c_void_p], C.c_char_p),
    ("rl_router_destroy", [C.c_void_p], None),
]

# multi-GPU router record sizes (include/rl_hip.h RL_ROUTE_*)
ROUTE_RECORD_BYTES = 32
ROUTE_REPLY_BYTES = 24
ROUTE_MAX_SHARDS = 16
ROUTE_LOCAL = 0xFFFFFFFF

_lib = None


def load_library(path: Optional[os.PathLike] = None) -> C.CDLL:
    """Load libratelimit_hip.so; raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"HIP extension not built: {p} missing (run __graft_entry__.build())")
    lib = C.CDLL(str(p))
    for name, argt, rest in ABI:
        # (a variant library given by path — an earlier round's build in a bench A/B — may lack
        # entry points added since; the in-tree library must export them all)
        f = getattr(lib, name) if path is None or hasattr(lib, name) else None
        if f is None:
            continue
        f.argtypes = argt
        f.restype = rest
    if path is None:
        _lib = lib
    return lib


class RedisError(RuntimeError):
    """redis.RedisError — the backend's only recoverable failure (service/ratelimit.go:276-281).
    `code` is the RL_E* return code when the error came from the C ABI."""

    def __init__(self, msg: str, code: Optional[int] = None):
        super().__init__(msg)
        self.code = code


# ---------------------------------------------------------------------------
# Flat batches (the C ABI's input layout)
# ---------------------------------------------------------------------------
@dataclass
class Batch:
    blob: np.ndarray      # uint8 key-prefix bytes
    off: np.ndarray       # uint32 [n_desc + 1]
    rule: np.ndarray      # uint32 [n_desc]
    req_of: np.ndarray    # uint32 [n_desc]
    now: np.ndarray       # int64 [n_req]
    hits: np.ndarray      # uint32 [n_req]
    # uint16 [n_desc] or None: EXPIRE jitter per descriptor, seconds (rl_batch.ttl_jitter;
    # JitterRand.Int63n(EXPIRATION_JITTER_MAX_SECONDS) drawn in serial order, fixed_cache_impl.go:69-72)
    jit: Optional[np.ndarray] = None

    @property
    def n_desc(self) -> int:
        return int(self.rule.shape[0])

    @property
    def n_req(self) -> int:
        return int(self.now.shape[0])

    def prefix(self, i: int) -> bytes:
        return bytes(self.blob[self.off[i]:self.off[i + 1]])

    def slice_requests(self, r0: int, r1: int) -> "Batch":
        """Requests [r0, r1) as their own batch."""
        d0 = int(np.searchsorted(self.req_of, r0, "left"))
        d1 = int(np.searchsorted(self.req_of, r1, "left"))
        b0, b1 = int(self.off[d0]), int(self.off[d1])
        return Batch(self.blob[b0:b1].copy(), (self.off[d0:d1 + 1] - b0).astype(np.uint32),
                     self.rule[d0:d1].copy(), (self.req_of[d0:d1] - r0).astype(np.uint32),
                     self.now[r0:r1].copy(), self.hits[r0:r1].copy(),
                     None if self.jit is None else self.jit[d0:d1].copy())


def cache_key_prefix(domain: str, entries: Sequence[tuple]) -> bytes:
    """GenerateCacheKey without the timestamp: domain '_' (key '_' value '_')*  (cache_key.go:57-65)."""
    out = bytearray(domain.encode())
    out += b"_"
    for k, v in entries:
        out += k.encode() + b"_" + v.encode() + b"_"
    return bytes(out)


def build_batch(requests: Sequence[tuple], jit=None) -> Batch:
    """requests: [(domain, [entries | None...], [rule_id...], hits_addend, now)] where each
    descriptor is a list of (key, value) and rule_id is NIL_RULE for a nil limit. jit: the
    EXPIRE jitter per descriptor (flat, serial order), or None."""
    blob = bytearray()
    off, rule, req_of, now, hits = [0], [], [], [], []
    for r, (domain, descs, rules, ha, t) in enumerate(requests):
        assert len(descs) == len(rules)
        for entries, rid in zip(descs, rules):
            if rid != NIL_RULE:
                blob += cache_key_prefix(domain, entries)
            off.append(len(blob))
            rule.append(rid)
            req_of.append(r)
        now.append(t)
        hits.append(ha)
    return Batch(np.frombuffer(bytes(blob), dtype=np.uint8).copy(), np.array(off, np.uint32),
                 np.array(rule, np.uint32), np.array(req_of, np.uint32), np.array(now, np.int64),
                 np.array(hits, np.uint32), None if jit is None else np.asarray(jit, np.uint16))


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


@dataclass
class CompactBatch:
    """A Batch in the compact host wire format (rl_batch_c): prefix bytes back to back, one word
    per descriptor (prefix length | rule id << 16), one per request (hits_addend | (now -
    now_base) << 24), req_of only when some request holds several descriptors."""
    blob: np.ndarray       # uint8
    desc_word: np.ndarray  # uint32 [n_desc]
    req_word: np.ndarray   # uint32 [n_req]
    req_of: Optional[np.ndarray]  # uint32 [n_desc] or None (one descriptor per request)
    now_base: int
    jit: Optional[np.ndarray] = None  # uint16 [n_desc] or None: EXPIRE jitter (rl_batch_c.ttl_jitter)

    @property
    def n_desc(self) -> int:
        return int(self.desc_word.shape[0])

    @property
    def n_req(self) -> int:
        return int(self.req_word.shape[0])

    @property
    def flags(self) -> int:
        return BC_ONE_PER_REQ if self.req_of is None else 0

    def struct(self) -> RlBatchC:
        s = RlBatchC()
        s.n_desc, s.n_req, s.blob_bytes, s.flags, s.now_base = (self.n_desc, self.n_req, int(self.blob.shape[0]),
                                                                self.flags, self.now_base)
        s.prefix_blob, s.desc_word, s.req_word = _ptr(self.blob), _ptr(self.desc_word), _ptr(self.req_word)
        s.req_of = 0 if self.req_of is None else _ptr(self.req_of)
        s.ttl_jitter = 0 if self.jit is None else _ptr(self.jit)
        return s

    def wire_bytes(self) -> int:
        """Bytes this batch moves host -> device (rl_submit_c's copies, without the blob slack)."""
        return (int(self.blob.shape[0]) + 4 * self.n_desc + 4 * self.n_req + (0 if self.req_of is None else 4 * self.n_desc)
                + (0 if self.jit is None else 2 * self.n_desc))


def compact_batch(b: Batch) -> CompactBatch:
    """Batch -> CompactBatch. Raises ValueError when the batch does not fit the compact form
    (rule id >= 0xFFFF, a prefix over 65535 bytes, hits_addend >= 2^24, times spanning > 255 s)."""
    lens = np.diff(b.off.astype(np.int64))
    if b.n_desc and (lens.max() > 0xFFFF or lens.min() < 0):
        raise ValueError("prefix length outside [0, 65535]")
    nil = b.rule == NIL_RULE
    if np.any(~nil & (b.rule >= NIL_RULE16)):
        raise ValueError("rule id >= 0xFFFF")
    # prefixes back to back: the compact form has no offsets, so the blob is rebuilt in order
    if b.n_desc and not (b.off[0] == 0 and b.off[-1] == b.blob.shape[0]):
        blob = np.concatenate([b.blob[b.off[i]:b.off[i + 1]] for i in range(b.n_desc)]).astype(np.uint8)
    else:
        blob = b.blob.copy()
    dw = (lens.astype(np.uint32) | (np.where(nil, NIL_RULE16, b.rule).astype(np.uint32) << 16)).astype(np.uint32)
    base = int(b.now.min()) if b.n_req else 0
    delta = b.now - base
    if b.n_req and (delta.max() > 255 or np.any(b.hits >= (1 << 24))):
        raise ValueError("request times span more than 255 s or hits_addend >= 2^24")
    rw = ((b.hits.astype(np.uint32) & 0xFFFFFF) | (delta.astype(np.uint32) << 24)).astype(np.uint32)
    one = b.n_desc == b.n_req and np.array_equal(b.req_of, np.arange(b.n_desc, dtype=np.uint32))
    return CompactBatch(blob, dw, rw, None if one else b.req_of.copy(), base,
                        None if b.jit is None else np.ascontiguousarray(b.jit, np.uint16))


def _batch_struct(b: Batch, ptrs=None) -> RlBatch:
    s = RlBatch()
    s.n_desc, s.n_req, s.blob_bytes, s.reserved = b.n_desc, b.n_req, int(b.blob.shape[0]), 0
    if ptrs is None:
        ptrs = [_ptr(b.blob), _ptr(b.off), _ptr(b.rule), _ptr(b.req_of), _ptr(b.now), _ptr(b.hits),
                0 if b.jit is None else _ptr(b.jit)]
    _set_ptrs(s, ptrs)
    return s


def _set_ptrs(s: RlBatch, ptrs):
    """blob, off, rule, req_of, now, hits[, ttl_jitter] into an rl_batch."""
    s.prefix_blob, s.prefix_off, s.rule_id, s.req_of, s.now, s.hits_addend = ptrs[:6]
    s.ttl_jitter = ptrs[6] if len(ptrs) > 6 and ptrs[6] else 0


# ---------------------------------------------------------------------------
# Engine (C ABI wrapper)
# ---------------------------------------------------------------------------
class Engine:
    def __init__(self, device: int = 0, log2_slots=(16, 16, 16, 14), near_limit_ratio: float = 0.8,
                 local_cache: bool = False, per_second_split: bool = False, max_batch_desc: int = 1 << 16,
                 max_batch_req: Optional[int] = None, max_blob_bytes: Optional[int] = None, sort_bits: int = 48,
                 hash_seed: int = 0x5EE7AB1E5EED, lib_path: Optional[os.PathLike] = None, lsd_only: bool = False,
                 pipeline: str = "v4", max_load_permille: int = 0, lag_window: bool = False):
        """pipeline: "v4" (default: tile-sorted records, hot keys decided in place, MSD buckets
        gathered and grouped in LDS) or "lsd" (radix-sort pipeline, also v4's fallback).
        lsd_only=True is pipeline="lsd". log2_slots: table slots per window generation for the
        key strings whose home unit is SECOND/MINUTE/HOUR/DAY."""
        if lsd_only:
            pipeline = "lsd"
        if pipeline not in PIPELINE_FLAGS:
            raise ValueError(f"pipeline must be one of {sorted(PIPELINE_FLAGS)}")
        self.lib = load_library(lib_path)
        cfg = RlConfig()
        cfg.struct_size = C.sizeof(RlConfig)
        cfg.device = device
        for i, v in enumerate(log2_slots):
            cfg.log2_slots[i] = v
        cfg.near_limit_ratio = near_limit_ratio
        cfg.local_cache = int(local_cache)
        cfg.per_second_split = int(per_second_split)
        cfg.max_batch_desc = max_batch_desc
        cfg.max_batch_req = max_batch_req or max_batch_desc
        cfg.max_blob_bytes = max_blob_bytes or max_batch_desc * 64
        cfg.sort_bits = sort_bits
        cfg.flags = PIPELINE_FLAGS[pipeline] | (CFG_LAG_WINDOW if lag_window else 0)
        cfg.hash_seed = hash_seed
        cfg.max_load_permille = max_load_permille
        self.cfg = cfg
        h = C.c_void_p()
        rc = self.lib.rl_create(C.byref(cfg), C.byref(h))
        if rc:
            raise RedisError(f"rl_create failed: {RL_ERRORS.get(rc, rc)}: "
                             f"{self.lib.rl_last_error(None).decode(errors='replace')}")
        self.h = h
        self.near_limit_ratio = near_limit_ratio

    def close(self):
        if getattr(self, "h", None):
            self.lib.rl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc:
            msg = self.lib.rl_last_error(self.h).decode()
            raise RedisError(f"{what}: {RL_ERRORS.get(rc, rc)}: {msg}", rc)

    def load_rules(self, rules: Sequence[tuple]):
        """rules: (requests_per_unit, unit) or (requests_per_unit, unit, shadow_mode)."""
        arr = (RlRule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            arr[i].requests_per_unit = r[0]
            arr[i].unit = r[1] | (RULE_SHADOW if len(r) > 2 and r[2] else 0)
        self._check(self.lib.rl_load_rules(self.h, arr, len(rules)), "rl_load_rules")

    def submit(self, b: Batch):
        """Host batch -> (status[n_desc] structured array, throttle_ms[n_req]); one batch in flight."""
        self.submit_host_async(b)
        return self.wait_into(b.n_desc, b.n_req)

    def submit_host_async(self, b: Batch):
        """rl_submit of a host batch with no output pointers: up to MAX_IN_FLIGHT in flight, the
        results wait in the engine's pinned memory until wait_into()."""
        s = _batch_struct(b)
        self._check(self.lib.rl_submit(self.h, C.byref(s), None, None), "rl_submit")

    def wait_into(self, n_desc: int, n_req: int):
        """rl_wait_into: complete the oldest batch, copying its results out."""
        out = np.zeros(n_desc, STATUS_DTYPE)
        thr = np.zeros(n_req, np.uint32)
        self._check(self.lib.rl_wait_into(self.h, _ptr(out) or None, _ptr(thr) or None), "rl_wait_into")
        return out, thr

    def wait_view(self, n_desc: int, n_req: int):
        """rl_wait_view: complete the oldest batch (a host batch submitted without output
        pointers) and return numpy views of its results in the slot's pinned memory (valid until
        the next submit)."""
        po, pt = C.c_void_p(), C.c_void_p()
        self._check(self.lib.rl_wait_view(self.h, C.byref(po), C.byref(pt)), "rl_wait_view")
        out = np.ctypeslib.as_array(C.cast(po, C.POINTER(C.c_uint8)), shape=(n_desc * STATUS_DTYPE.itemsize,))
        thr = np.ctypeslib.as_array(C.cast(pt, C.POINTER(C.c_uint32)), shape=(n_req,))
        return out.view(STATUS_DTYPE), thr

    def host_acquire(self) -> dict:
        """rl_host_acquire: numpy views of the next free pinned staging slot (zero-copy submit).
        The views of a slot are built once and reused (the slots rotate; a batcher's loop should
        not pay for six ctypes casts per batch)."""
        hb = RlHostBatch()
        self._check(self.lib.rl_host_acquire(self.h, C.byref(hb)), "rl_host_acquire")
        cache = self.__dict__.setdefault("_slot_views", {})
        got = cache.get(hb.prefix_blob)
        if got is not None:
            return got

        def view(ptr, n, dt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
        got = dict(blob=view(hb.prefix_blob, hb.max_blob, np.uint8), off=view(hb.prefix_off, hb.max_desc + 1, np.uint32),
                   rule=view(hb.rule_id, hb.max_desc, np.uint32), req_of=view(hb.req_of, hb.max_desc, np.uint32),
                   now=view(hb.now, hb.max_req, np.int64), hits=view(hb.hits_addend, hb.max_req, np.uint32),
                   jit=view(hb.ttl_jitter, hb.max_desc, np.uint16))
        cache[hb.prefix_blob] = got
        return got

    def submit_staged(self, n_desc: int, n_req: int, blob_bytes: int, staged: dict, jitter: bool = False):
        """rl_submit of a batch built in place in an acquired staging slot (no host copy);
        jitter: the slot's jitter array holds the batch's EXPIRE jitter."""
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        s.prefix_blob, s.prefix_off, s.rule_id, s.req_of, s.now, s.hits_addend = (
            staged[k].ctypes.data for k in ("blob", "off", "rule", "req_of", "now", "hits"))
        s.ttl_jitter = staged["jit"].ctypes.data if jitter else 0
        self._check(self.lib.rl_submit(self.h, C.byref(s), None, None), "rl_submit")

    # ---- compact host batches (rl_batch_c, raw replies) ----
    def submit_c(self, cb: CompactBatch):
        """rl_submit_c of a compact host batch (copied into the staging slot)."""
        s = cb.struct()
        self._check(self.lib.rl_submit_c(self.h, C.byref(s)), "rl_submit_c")

    def host_acquire_c(self) -> dict:
        """rl_host_acquire_c: numpy views of the next free slot in the compact layout (built once
        per slot)."""
        hb = RlHostBatchC()
        self._check(self.lib.rl_host_acquire_c(self.h, C.byref(hb)), "rl_host_acquire_c")
        cache = self.__dict__.setdefault("_slot_views_c", {})
        got = cache.get(hb.prefix_blob)
        if got is not None:
            return got

        def view(ptr, n, dt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
        got = dict(blob=view(hb.prefix_blob, hb.max_blob, np.uint8), desc_word=view(hb.desc_word, hb.max_desc, np.uint32),
                   req_word=view(hb.req_word, hb.max_req, np.uint32), req_of=view(hb.req_of, hb.max_desc, np.uint32),
                   jit=view(hb.ttl_jitter, hb.max_desc, np.uint16))
        cache[hb.prefix_blob] = got
        return got

    def submit_c_staged(self, n_desc: int, n_req: int, blob_bytes: int, now_base: int, staged: dict,
                        one_per_req: bool = True, jitter: bool = False):
        """rl_submit_c of a compact batch built in place in an acquired slot (no host copy)."""
        s = RlBatchC()
        s.n_desc, s.n_req, s.blob_bytes, s.now_base = n_desc, n_req, blob_bytes, now_base
        s.flags = BC_ONE_PER_REQ if one_per_req else 0
        s.prefix_blob, s.desc_word, s.req_word = (staged[k].ctypes.data for k in ("blob", "desc_word", "req_word"))
        s.req_of = 0 if one_per_req else staged["req_of"].ctypes.data
        s.ttl_jitter = staged["jit"].ctypes.data if jitter else 0
        self._check(self.lib.rl_submit_c(self.h, C.byref(s)), "rl_submit_c")

    def wait_raw_view(self, n_desc: int) -> np.ndarray:
        """rl_wait_raw_view: the oldest compact batch's raw replies in the slot (RAW_DTYPE view)."""
        p = C.c_void_p()
        self._check(self.lib.rl_wait_raw_view(self.h, C.byref(p)), "rl_wait_raw_view")
        if not n_desc:
            return np.zeros(0, RAW_DTYPE)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n_desc * 8,)).view(RAW_DTYPE)

    def wait_raw_into(self, n_desc: int) -> np.ndarray:
        out = np.zeros(n_desc, RAW_DTYPE)
        self._check(self.lib.rl_wait_raw_into(self.h, _ptr(out) or None), "rl_wait_raw_into")
        return out

    def decide_raw(self, cb: CompactBatch, raw: np.ndarray, d0: int = 0, d1: Optional[int] = None,
                   out: Optional[np.ndarray] = None, thr: Optional[np.ndarray] = None):
        """rl_decide_raw: statuses and ThrottleMillis of descriptors [d0, d1) from raw replies."""
        d1 = cb.n_desc if d1 is None else d1
        out = np.zeros(cb.n_desc, STATUS_DTYPE) if out is None else out
        thr = np.zeros(cb.n_req, np.uint32) if thr is None else thr
        s = cb.struct()
        self._check(self.lib.rl_decide_raw(self.h, C.byref(s), _ptr(raw), d0, d1, _ptr(out) or None,
                                           _ptr(thr) or None), "rl_decide_raw")
        return out, thr

    def submit_compact(self, b: Batch):
        """A host batch through the compact wire format: rl_submit_c, rl_wait_raw_into,
        rl_decide_raw -> (statuses, throttles), equal to submit(b)."""
        cb = compact_batch(b)
        self.submit_c(cb)
        raw = self.wait_raw_into(cb.n_desc)
        return self.decide_raw(cb, raw)

    def occupancy(self) -> dict:
        o = RlOccupancy()
        self._check(self.lib.rl_get_occupancy(self.h, C.byref(o)), "rl_get_occupancy")
        return {k: list(getattr(o, k)) for k in ("gen", "live", "limit", "slots")}

    def submit_device_async(self, n_desc: int, n_req: int, blob_bytes: int, ptrs, out_ptr: int, thr_ptr: int):
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        _set_ptrs(s, ptrs)
        self._check(self.lib.rl_submit_device(self.h, C.byref(s), out_ptr, thr_ptr), "rl_submit_device")

    @staticmethod
    def device_batch(n_desc: int, n_req: int, blob_bytes: int, ptrs) -> RlBatch:
        """An rl_batch of device pointers (ptrs = blob, off, rule, req_of, now, hits[, ttl_jitter])."""
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        _set_ptrs(s, ptrs)
        return s

    def submit_pipelined(self, n_desc: int, n_req: int, blob_bytes: int, ptrs, out_ptr: int, thr_ptr: int):
        """Device batch with complete inputs, behind at most one batch in flight (rl_submit_pipelined):
        wait() completes the oldest. The two in-flight batches need distinct output buffers."""
        self.submit_pipelined_batch(self.device_batch(n_desc, n_req, blob_bytes, ptrs), out_ptr, thr_ptr)

    def submit_pipelined_batch(self, s: RlBatch, out_ptr: int, thr_ptr: int):
        """submit_pipelined with a prebuilt device_batch() (no per-call marshalling)."""
        self._check(self.lib.rl_submit_pipelined(self.h, C.byref(s), out_ptr, thr_ptr), "rl_submit_pipelined")

    def wait(self):
        self._check(self.lib.rl_wait(self.h), "rl_wait")

    def query(self) -> bool:
        """rl_query: True when the oldest batch in flight is done on the device."""
        rc = self.lib.rl_query(self.h)
        if rc < 0:
            self._check(rc, "rl_query")
        return rc == 1

    def load_tree(self, nodes: np.ndarray, names: bytes):
        """nodes: uint32 [n, 4] (parent, name_off, name_len, rule); names: the tree's map keys."""
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32).reshape(-1, 4)
        nb = np.frombuffer(bytes(names) or b"\0", np.uint8)
        self._check(self.lib.rl_load_tree(self.h, nodes.ctypes.data_as(C.POINTER(RlTreeNode)), nodes.shape[0],
                                          nb.ctypes.data, len(names)), "rl_load_tree")

    def resolve_device(self, s: "RlResolveBatch", d_rule_out: int):
        """rl_resolve_device: an rl_resolve_batch of device pointers -> rule ids in device memory,
        ordered before the next submit."""
        self._check(self.lib.rl_resolve_device(self.h, C.byref(s), d_rule_out), "rl_resolve_device")

    def resolve(self, rb) -> np.ndarray:
        """GetLimit for every descriptor of an rl_config.ResolveBatch -> rule id per descriptor."""
        out = np.zeros(max(1, rb.n_desc), np.uint32)
        s = rb.struct()
        self._check(self.lib.rl_resolve(self.h, C.byref(s), _ptr(out)), "rl_resolve")
        return out[:rb.n_desc]

    def reset(self):
        self._check(self.lib.rl_reset(self.h), "rl_reset")

    def stats(self) -> dict:
        s = RlEngineStats()
        self._check(self.lib.rl_get_stats(self.h, C.byref(s)), "rl_get_stats")
        return {k: getattr(s, k) for k, _ in RlEngineStats._fields_}

    def set_timing(self, on: bool):
        self._check(self.lib.rl_set_timing(self.h, int(on)), "rl_set_timing")

    def kernel_times(self) -> dict:
        cap = 32
        names = (C.c_char_p * cap)()
        ms = (C.c_double * cap)()
        cnt = (C.c_uint64 * cap)()
        n = C.c_uint32()
        self._check(self.lib.rl_kernel_times(self.h, names, ms, cnt, cap, C.byref(n)), "rl_kernel_times")
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(n.value)}

    def last_batch_info(self) -> dict:
        v = [C.c_uint64() for _ in range(4)]
        self._check(self.lib.rl_last_batch_info(self.h, *[C.byref(x) for x in v]), "rl_last_batch_info")
        return dict(zip(["unique_keys", "n_desc", "n_req", "blob_bytes"], [x.value for x in v]))

    def stream(self) -> int:
        return self.lib.rl_stream(self.h) or 0

    def set_stream(self, hip_stream: int):
        """Order the engine's work on an external HIP stream (0 = the engine's own)."""
        self._check(self.lib.rl_set_stream(self.h, hip_stream or None), "rl_set_stream")

    # -- multi-GPU router (include/rl_hip.h, "Multi-GPU router") -----------------------
    def route_pack(self, n_desc: int, n_req: int, blob_bytes: int, ptrs, origin: int, n_shards: int, send_ptr: int,
                   send_counts_ptr: int, perm_ptr: int) -> list:
        """Device batch -> routed records grouped by owner; returns the per-owner counts."""
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        _set_ptrs(s, ptrs)
        counts = (C.c_uint32 * n_shards)()
        self._check(self.lib.rl_route_pack(self.h, C.byref(s), origin, n_shards, send_ptr, send_counts_ptr, perm_ptr,
                                           counts), "rl_route_pack")
        return list(counts)

    def route_pack_async(self, n_desc: int, n_req: int, blob_bytes: int, ptrs, origin: int, n_shards: int,
                         send_ptr: int, x_ptr: int, perm_ptr: int):
        """rl_route_pack without the host round trip: (count, status) per owner in x (device)."""
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        _set_ptrs(s, ptrs)
        self._check(self.lib.rl_route_pack_async(self.h, C.byref(s), origin, n_shards, send_ptr, x_ptr, perm_ptr),
                    "rl_route_pack_async")

    def route_pack_strided(self, n_desc: int, n_req: int, blob_bytes: int, ptrs, origin: int, n_shards: int,
                           stride: int, send_ptr: int, x_ptr: int, perm_ptr: int):
        """rl_route_pack_strided: one-kernel pack, owner j's records at send[j * stride ...]."""
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, blob_bytes, 0
        _set_ptrs(s, ptrs)
        self._check(self.lib.rl_route_pack_strided(self.h, C.byref(s), origin, n_shards, stride, send_ptr, x_ptr,
                                                   perm_ptr), "rl_route_pack_strided")

    def submit_routed_async(self, rec_ptr: int, n: int, reply_ptr: int):
        self._check(self.lib.rl_submit_routed(self.h, rec_ptr, n, reply_ptr), "rl_submit_routed")

    def route_unpack(self, n_desc: int, n_req: int, req_of_ptr: int, perm_ptr: int, reply_ptr: int, out_ptr: int,
                     thr_ptr: int):
        s = RlBatch()
        s.n_desc, s.n_req, s.blob_bytes, s.reserved = n_desc, n_req, 0, 0
        s.req_of = req_of_ptr
        self._check(self.lib.rl_route_unpack(self.h, C.byref(s), perm_ptr, reply_ptr, out_ptr, thr_ptr),
                    "rl_route_unpack")


class Router:
    """The routed step owned by the C ABI (rl_router_*): G engines in this process (local
    transport) or this rank's engine over an RCCL communicator (rccl_id from
    router_unique_id() on one rank, shared out of band). combine: hot-prefix combining
    (DESIGN.md §5); host: pinned host staging for submit_host / wait_into."""

    def __init__(self, engines, max_desc: int, n_shards: Optional[int] = None, rank: int = 0,
                 rccl_id: Optional[bytes] = None, combine: bool = True, host: bool = False,
                 max_blob_bytes: int = 0, emulated: bool = False, host_xchg=None):
        """emulated: rccl_id is an emu_world() id — the collective transport with in-process
        collectives (one Router per rank, each driven by its own thread)."""
        self.lib = engines[0].lib
        self.engines = list(engines)
        cfg = RlRouterConfig()
        cfg.struct_size = C.sizeof(RlRouterConfig)
        cfg.n_shards = n_shards if n_shards is not None else len(engines)
        cfg.rank = rank
        cfg.max_desc = max_desc
        cfg.flags = ((0 if combine else ROUTER_NO_COMBINE) | (ROUTER_HOST if host else 0)
                     | (ROUTER_EMULATED if emulated else 0) | (ROUTER_HOST_XCHG if host_xchg is not None else 0))
        self._xchg = None
        if host_xchg is not None:  # a HOST_XCHG_FN the caller keeps alive as long as the router
            self._xchg = host_xchg
            self.lib.rl_router_use_host_xchg(C.cast(host_xchg, C.c_void_p), None)
        cfg.max_blob_bytes = max_blob_bytes
        self._id = None
        if rccl_id is not None:
            self._id = C.create_string_buffer(bytes(rccl_id), ROUTER_ID_BYTES)
            cfg.rccl_id = C.cast(self._id, C.c_void_p)
        arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
        self.h = C.c_void_p()
        rc = self.lib.rl_router_create(C.byref(cfg), arr, C.byref(self.h))
        if rc:
            raise RedisError(f"rl_router_create failed: {RL_ERRORS.get(rc, rc)}", rc)
        self.n = len(engines)
        self._keep = []  # ctypes arrays of steps in flight

    @staticmethod
    def unique_id(lib=None) -> bytes:
        lib = lib or load_library()
        buf = C.create_string_buffer(ROUTER_ID_BYTES)
        rc = lib.rl_router_unique_id(buf)
        if rc:
            raise RedisError(f"rl_router_unique_id: {RL_ERRORS.get(rc, rc)}")
        return buf.raw

    @staticmethod
    def emu_world(n_ranks: int, lib=None) -> bytes:
        """rl_router_emu_world: the id of an in-process world of n_ranks emulated ranks."""
        lib = lib or load_library()
        buf = C.create_string_buffer(ROUTER_ID_BYTES)
        rc = lib.rl_router_emu_world(n_ranks, buf)
        if rc:
            raise RedisError(f"rl_router_emu_world: {RL_ERRORS.get(rc, rc)}", rc)
        return buf.raw

    def _check(self, rc, what):
        if rc:
            raise RedisError(f"{what}: {RL_ERRORS.get(rc, rc)}: {self.lib.rl_router_last_error(self.h).decode()}", rc)

    def step(self, batches, out_ptrs, thr_ptrs):
        """batches: RlBatch per engine (device pointers); outputs: device pointers per engine."""
        arr = (RlBatch * self.n)(*batches)
        o = (C.c_void_p * self.n)(*out_ptrs)
        t = (C.c_void_p * self.n)(*thr_ptrs)
        self._check(self.lib.rl_router_step(self.h, arr, o, t), "rl_router_step")

    def submit(self, batches, out_ptrs, thr_ptrs):
        """rl_router_submit: a step handed over, up to three in flight (wait() completes the oldest)."""
        arr = (RlBatch * self.n)(*batches)
        o = (C.c_void_p * self.n)(*out_ptrs)
        t = (C.c_void_p * self.n)(*thr_ptrs)
        self._keep.append((arr, o, t))
        self._check(self.lib.rl_router_submit(self.h, arr, o, t), "rl_router_submit")

    def wait(self):
        try:
            self._check(self.lib.rl_router_wait(self.h), "rl_router_wait")
        finally:
            if self._keep:
                self._keep.pop(0)

    def host_acquire(self, shard: int = 0) -> dict:
        """rl_router_host_acquire: numpy views of the next step's pinned staging slot of a shard."""
        hb = RlHostBatch()
        self._check(self.lib.rl_router_host_acquire(self.h, shard, C.byref(hb)), "rl_router_host_acquire")

        def view(ptr, n, dt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
        return dict(blob=view(hb.prefix_blob, hb.max_blob, np.uint8), off=view(hb.prefix_off, hb.max_desc + 1, np.uint32),
                    rule=view(hb.rule_id, hb.max_desc, np.uint32), req_of=view(hb.req_of, hb.max_desc, np.uint32),
                    now=view(hb.now, hb.max_req, np.int64), hits=view(hb.hits_addend, hb.max_req, np.uint32))

    def submit_host(self, batches):
        """rl_router_submit_host: host Batch objects (or dicts from host_acquire with n_desc/n_req/blob_bytes)."""
        structs = []
        for b in batches:
            if isinstance(b, dict):
                s = RlBatch()
                s.n_desc, s.n_req, s.blob_bytes, s.reserved = b["n_desc"], b["n_req"], b["blob_bytes"], 0
                s.prefix_blob, s.prefix_off, s.rule_id, s.req_of, s.now, s.hits_addend = (
                    b[k].ctypes.data for k in ("blob", "off", "rule", "req_of", "now", "hits"))
                structs.append(s)
            else:
                structs.append(_batch_struct(b))
        arr = (RlBatch * self.n)(*structs)
        self._keep.append((arr, batches))
        self._check(self.lib.rl_router_submit_host(self.h, arr), "rl_router_submit_host")

    def wait_into(self, sizes):
        """rl_router_wait_into: sizes = [(n_desc, n_req)] per shard -> [(status array, throttle array)]."""
        outs = [np.zeros(max(1, nd), STATUS_DTYPE) for nd, _ in sizes]
        thrs = [np.zeros(max(1, nr), np.uint32) for _, nr in sizes]
        o = (C.c_void_p * self.n)(*[x.ctypes.data for x in outs])
        t = (C.c_void_p * self.n)(*[x.ctypes.data for x in thrs])
        try:
            self._check(self.lib.rl_router_wait_into(self.h, o, t), "rl_router_wait_into")
        finally:
            if self._keep:
                self._keep.pop(0)
        return [(outs[i][:nd], thrs[i][:nr]) for i, (nd, nr) in enumerate(sizes)]

    def allgather_host(self, data: bytes, n_ranks: int) -> list:
        """rl_router_allgather_host: every rank's `data` (the same length everywhere), in rank
        order (the batchers' rule and stop agreement)."""
        buf = C.create_string_buffer(bytes(data), max(1, len(data)))
        out = C.create_string_buffer(max(1, len(data) * n_ranks))
        self._check(self.lib.rl_router_allgather_host(self.h, buf, len(data), out), "rl_router_allgather_host")
        raw = out.raw
        return [raw[i * len(data):(i + 1) * len(data)] for i in range(n_ranks)]

    def stats(self) -> dict:
        s = RlRouterStats()
        self.lib.rl_router_get_stats(self.h, C.byref(s))
        d = {k: getattr(s, k) for k, _ in RlRouterStats._fields_}
        for k in ("status", "recv", "sent"):
            d[k] = list(d[k])[:s.n_shards]
        return d

    def close(self):
        if self.h:
            self.lib.rl_router_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


# ---------------------------------------------------------------------------
# Mirror of the reference's RateLimitCache contract (for reference-style tests)
# ---------------------------------------------------------------------------
class Counter:
    def __init__(self):
        self.v = 0

    def Add(self, d: int):
        self.v += int(d)

    def Value(self) -> int:
        return self.v


@dataclass
class RateLimitStats:
    TotalHits: Counter = field(default_factory=Counter)
    OverLimit: Counter = field(default_factory=Counter)
    NearLimit: Counter = field(default_factory=Counter)
    OverLimitWithLocalCache: Counter = field(default_factory=Counter)
    ShadowMode: Counter = field(default_factory=Counter)  # extension (RULE_SHADOW)


class StatsStore:
    """Counters shared by name, like gostats' NewCounter (config_impl.go:64-71)."""

    def __init__(self):
        self.m = {}

    def get(self, key: str) -> RateLimitStats:
        return self.m.setdefault(key, RateLimitStats())


@dataclass(frozen=True)
class RateLimitLimit:
    RequestsPerUnit: int
    Unit: int


@dataclass
class RateLimit:
    FullKey: str
    Stats: RateLimitStats
    Limit: RateLimitLimit
    SleepOnThrottle: bool = False
    ReportDetails: bool = False
    ShadowMode: bool = False  # extension: the fork's config has no shadow_mode (config_impl.go:49-59)


def NewRateLimit(requests_per_unit: int, unit: int, key: str, scope: StatsStore, sleep_on_throttle=False,
                 report_details=False, shadow_mode=False) -> RateLimit:
    """config.NewRateLimit  src/config/config_impl.go:79-89 (+ shadow_mode, an extension)"""
    return RateLimit(key, scope.get(key), RateLimitLimit(requests_per_unit, unit), sleep_on_throttle, report_details,
                     shadow_mode)


@dataclass
class RateLimitRequest:
    Domain: str
    Descriptors: list  # list of list of (key, value)
    HitsAddend: int = 1


def NewRateLimitRequest(domain: str, descriptors, hits_addend: int) -> RateLimitRequest:
    """test/common/common.go NewRateLimitRequest"""
    return RateLimitRequest(domain, [list(d) for d in descriptors], hits_addend)


@dataclass(frozen=True)
class DescriptorStatus:
    Code: int
    CurrentLimit: Optional[RateLimitLimit]
    LimitRemaining: int
    DurationUntilReset: Optional[int] = None


@dataclass
class DoLimitResponse:
    DescriptorStatuses: list
    ThrottleMillis: int = 0


def CalculateReset(limit: RateLimitLimit, now: int) -> int:
    """utils.CalculateReset  src/utils/utilities.go:34-38"""
    d = UNIT_DIVIDER[limit.Unit]
    return d - now % d


class HipRateLimitCache:
    """limiter.RateLimitCache on the HIP engine. do_limit() is DoLimit for one request;
    do_limit_batch() submits several requests as ONE device batch in serial order."""

    def __init__(self, time_source, local_cache: bool = False, near_limit_ratio: float = 0.8,
                 per_second_split: bool = False, **engine_kw):
        self.time_source = time_source
        self.engine = Engine(near_limit_ratio=near_limit_ratio, local_cache=local_cache,
                             per_second_split=per_second_split, **engine_kw)
        self.rule_ids = {}
        self.rules = []
        self.dirty = False

    def _rule(self, lim: RateLimitLimit, shadow: bool = False) -> int:
        k = (lim.RequestsPerUnit, lim.Unit, bool(shadow))
        if k not in self.rule_ids:
            self.rule_ids[k] = len(self.rules)
            self.rules.append(k)
            self.dirty = True
        return self.rule_ids[k]

    def DoLimit(self, request: RateLimitRequest, limits: list) -> DoLimitResponse:
        return self.do_limit_batch([(request, limits)])[0]

    def Flush(self):
        pass

    def do_limit_batch(self, calls) -> list:
        reqs = []
        nows = []
        for request, limits in calls:
            assert len(request.Descriptors) == len(limits), "assert: len(request.Descriptors) == len(limits)"
            now = self.time_source()
            nows.append(now)
            h = max(1, request.HitsAddend)
            rules = []
            for lim in limits:
                if lim is None:
                    rules.append(NIL_RULE)
                else:
                    rules.append(self._rule(lim.Limit, lim.ShadowMode))
                    lim.Stats.TotalHits.Add(h)  # base_limiter.go:49-51
            reqs.append((request.Domain, request.Descriptors, rules, request.HitsAddend, now))
        if self.dirty:
            self.engine.load_rules(self.rules)
            self.dirty = False
        st, thr = self.engine.submit(build_batch(reqs))
        out = []
        d = 0
        for r, (request, limits) in enumerate(calls):
            sts = []
            for lim in limits:
                s = st[d]
                d += 1
                code = int(s["code_flags"]) & 0xFF
                fl = int(s["code_flags"]) >> 8
                if lim is None or not fl & FLAG_HAS_LIMIT:
                    sts.append(DescriptorStatus(code, None, int(s["limit_remaining"])))
                    continue
                sts.append(DescriptorStatus(code, lim.Limit, int(s["limit_remaining"]), int(s["reset_s"])))
                lim.Stats.OverLimit.Add(int(s["over_limit_delta"]))
                if fl & FLAG_LOCAL_CACHE_HIT:
                    lim.Stats.OverLimitWithLocalCache.Add(int(s["over_limit_delta"]))
                lim.Stats.NearLimit.Add(int(s["near_limit_delta"]))
                if fl & FLAG_SHADOW:
                    lim.Stats.ShadowMode.Add(1)
            out.append(DoLimitResponse(sts, int(thr[r])))
        return out

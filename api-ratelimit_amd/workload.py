"""Synthetic request streams for BASELINE.json configs 1-5.

Deterministic and vectorised (numpy): a counter-based splitmix64 generator, bounded
Zipf sampling by rejection-inversion (Hörmann & Derflinger 1996), a fixed bijective
permutation of ranks so hot keys are not adjacent, and vectorised construction of the
key-prefix blob (GenerateCacheKey's "domain_k1_v1_..._" bytes, cache_key.go:57-65).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from hiprl import Batch, DAY, HOUR, MINUTE, SECOND

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of (x + golden) — counter-based: value i of stream s is
    splitmix64(s * 2^40 + i)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(seed: int, stream: int, start: int, n: int) -> np.ndarray:
    ctr = np.arange(start, start + n, dtype=np.uint64) + np.uint64(((seed * 1000003 + stream) & 0xFFFFFF) << 40)
    return (splitmix64(ctr) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


class Zipf:
    """Bounded Zipf(s) on ranks 1..N by rejection-inversion (exact distribution)."""

    def __init__(self, N: int, s: float):
        self.N, self.s = N, s
        self.hx1 = self.H(1.5) - 1.0
        self.hN = self.H(N + 0.5)
        self.sq = 2.0 - self.Hinv(self.H(2.5) - self.h(2.0))

    def h(self, x):
        return np.exp(-self.s * np.log(x))

    def H(self, x):
        lx = np.log(x)
        t = (1.0 - self.s) * lx
        return lx * np.where(np.abs(t) > 1e-8, np.expm1(t) / np.where(t == 0, 1, t), 1 + t / 2)

    def Hinv(self, x):
        t = x * (1.0 - self.s)
        t = np.maximum(t, -1.0 + 1e-16)
        return np.exp(np.where(np.abs(t) > 1e-8, np.log1p(t) / np.where(t == 0, 1, t), 1 - t / 2) * x)

    def sample(self, seed: int, stream: int, n: int) -> np.ndarray:
        out = np.empty(n, np.int64)
        todo = np.arange(n)
        draw = 0
        while todo.size:
            u = uniform01(seed, stream, draw, todo.size)
            draw += todo.size
            u = self.hN + u * (self.hx1 - self.hN)
            x = self.Hinv(u)
            k = np.clip(np.floor(x + 0.5), 1, self.N)
            ok = (k - x <= self.sq) | (u >= self.H(k + 0.5) - self.h(k))
            out[todo[ok]] = k[ok].astype(np.int64)
            todo = todo[~ok]
        return out


def permute(rank: np.ndarray, N: int) -> np.ndarray:
    """Bijection of [0, N): affine map with a multiplier coprime to N."""
    a = 2654435761
    while math.gcd(a, N) != 1:
        a += 2
    return ((rank.astype(np.uint64) * np.uint64(a) + np.uint64(0x2545F491)) % np.uint64(N)).astype(np.uint64)


def _ndigits(v: np.ndarray) -> np.ndarray:
    d = np.ones(v.shape, np.int64)
    t = v.copy()
    for _ in range(20):
        t = t // np.uint64(10)
        nz = t > 0
        if not nz.any():
            break
        d += nz
    return d


def prefix_blob(parts) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate per-descriptor fields: each part is bytes (same for all) or a uint64
    array rendered in decimal. Returns (blob uint8, off uint32[n+1])."""
    n = next(len(p) for p in parts if not isinstance(p, (bytes, bytearray)))
    lens = np.zeros(n, np.int64)
    meta = []
    for p in parts:
        if isinstance(p, (bytes, bytearray)):
            lens += len(p)
            meta.append(("b", p, None))
        else:
            nd = _ndigits(p)
            lens += nd
            meta.append(("d", p, nd))
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    blob = np.zeros(int(off[-1]) + 32, np.uint8)  # slack for the device's 8-byte word reads
    cur = off[:-1].copy()
    for kind, p, nd in meta:
        if kind == "b":
            for j, ch in enumerate(p):
                blob[cur + j] = ch
            cur += len(p)
        else:
            v = p.astype(np.uint64).copy()
            maxd = int(nd.max())
            for j in range(maxd):  # least-significant digit first, written right to left
                pos = cur + nd - 1 - j
                m = j < nd
                blob[pos[m]] = (v[m] % np.uint64(10)).astype(np.uint8) + 48
                v //= np.uint64(10)
            cur += nd
    return blob, off.astype(np.uint32)


@dataclass
class Workload:
    name: str
    rules: list
    batches: list  # list of Batch
    note: str


def config3_batch(b: int, d: int = 1_000_000, N: int = 100_000_000, s: float = 1.1, seed: int = 3,
                  t0: int = 1_700_000_000, batches_per_s: int = 1) -> Batch:
    """Config 3: 1e8 keys Zipf(1.1), ranks through a fixed permutation, rule by rank % 3
    (SECOND 10 / MINUTE 600 / HOUR 36000), 1 descriptor per request, h = 1,
    now = t0 + b // batches_per_s."""
    z = Zipf(N, s)
    rank = z.sample(seed, b, d) - 1
    key = permute(rank, N)
    rule = (rank % 3).astype(np.uint32)
    blob, off = prefix_blob([b"bench_k_", key, b"_"])
    return Batch(blob, off, rule, np.arange(d, dtype=np.uint32), np.full(d, t0 + b // batches_per_s, np.int64),
                 np.ones(d, np.uint32))


CONFIG3_RULES = [(10, SECOND), (600, MINUTE), (36000, HOUR)]


def config2_batch(b: int, d: int = 1_000_000, N: int = 1_000_000, seed: int = 2, t0: int = 1_700_000_000,
                  batches_per_s: int = 1) -> Batch:
    """Config 2: 1e6 uniform keys, SECOND L=5, 1 descriptor per request, now = t0 + b // batches_per_s."""
    u = uniform01(seed, b, 0, d)
    rank = np.minimum((u * N).astype(np.int64), N - 1)
    blob, off = prefix_blob([b"bench_k_", permute(rank, N), b"_"])
    return Batch(blob, off, np.zeros(d, np.uint32), np.arange(d, dtype=np.uint32),
                 np.full(d, t0 + b // batches_per_s, np.int64), np.ones(d, np.uint32))


CONFIG2_RULES = [(5, SECOND)]


def config1_batch(b: int, d: int = 10_000, seed: int = 1, t0: int = 1_700_000_000) -> Batch:
    """Config 1 (examples/ratelimit/config): 10k keys [("foo","u<i>"),("baz","x")] ->
    rl.foo.baz SECOND 1 (example.yaml:12-29) and mongo_cps database users/default SECOND 500
    (config.yaml:2-14); 1 descriptor per request, h = 1, uniform i, now = t0 + b."""
    u = uniform01(seed, b, 0, d)
    i = np.minimum((u * 10_000).astype(np.int64), 9_999).astype(np.uint64)
    mongo = uniform01(seed, 1000 + b, 0, d) < 0.1
    blob_a, off_a = prefix_blob([b"rl_foo_u", i, b"_baz_x_"])
    users = uniform01(seed, 2000 + b, 0, d) < 0.5
    # build mixed blob row by row (small config)
    parts, offs = [], [0]
    for k in range(d):
        if mongo[k]:
            p = b"mongo_cps_database_users_" if users[k] else b"mongo_cps_database_default_"
        else:
            p = bytes(blob_a[off_a[k]:off_a[k + 1]])
        parts.append(p)
        offs.append(offs[-1] + len(p))
    blob = np.frombuffer(b"".join(parts) + b"\0" * 32, np.uint8).copy()
    rule = np.where(mongo, 1, 0).astype(np.uint32)
    return Batch(blob, np.array(offs, np.uint32), rule, np.arange(d, dtype=np.uint32),
                 np.full(d, t0 + b, np.int64), np.ones(d, np.uint32))


CONFIG1_RULES = [(1, SECOND), (500, SECOND)]


def algorithmic_bytes(batch: Batch, unique_keys: int) -> int:
    """Σ(len(prefix) + 4 off + 4 rule + 4 req) + r·(8 now + 4 h) + 20·d + 4·r + 64·U."""
    d, r = batch.n_desc, batch.n_req
    prefix = int(batch.off[-1]) - int(batch.off[0])
    return prefix + 12 * d + 12 * r + 20 * d + 4 * r + 64 * unique_keys


# ---------------------------------------------------------------------------------------
# Config 4: nested 4-entry descriptors matched by a synthetic 4-level YAML tree
# (GetLimit semantics, config_impl.go:274-323), resolved on the device (rl_resolve).
# ---------------------------------------------------------------------------------------
CONFIG4_KEYS = ("a", "b", "c", "d")
CONFIG4_UNITS = ("second", "minute", "hour", "day")


def config4_yaml(seed: int = 4, fan: int = 6, domain: str = "bench4") -> str:
    """A seeded 4-level descriptor tree in the reference's YAML schema: at each level a
    key-only default node (most of the time) and `fan` key/value nodes; limits at random
    depths (always on level-4 defaults), some nodes whitelisted (no limit)."""
    rng = np.random.default_rng(seed)
    lines = [f"domain: {domain}", "descriptors:"]

    def node(level: int, value, ind: str):
        lines.append(f"{ind}- key: {CONFIG4_KEYS[level]}")
        if value is not None:
            lines.append(f'{ind}  value: "{value}"')
        if (level == 3 and value is None) or rng.random() < 0.45:
            lines.append(f"{ind}  rate_limit:")
            lines.append(f"{ind}    unit: {CONFIG4_UNITS[int(rng.integers(0, 3))]}")
            lines.append(f"{ind}    requests_per_unit: {int(rng.integers(1, 50))}")
        if level < 3:
            lines.append(f"{ind}  descriptors:")
            children(level + 1, ind + "    ")

    def children(level: int, ind: str):
        if rng.random() < 0.85:
            node(level, None, ind)
        for v in range(fan):
            if rng.random() < 0.8:
                node(level, v, ind)

    children(0, "  ")
    return "\n".join(lines) + "\n"


def config4_descriptors(seed: int, n: int, fan: int = 6, values: int = 1000, domain: str = "bench4"):
    """n descriptors [(domain, [(key, value)...])]: mostly 4 entries a,b,c,d with values that
    hit the tree's key/value nodes (< fan) or fall back to its defaults; some shorter, some
    with a foreign key or an unknown domain."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        ne = 4 if rng.random() < 0.8 else int(rng.integers(1, 4))
        ents = []
        for lv in range(ne):
            key = CONFIG4_KEYS[lv] if rng.random() < 0.97 else "x"
            v = int(rng.integers(0, fan)) if rng.random() < 0.5 else int(rng.integers(0, values))
            ents.append((key, str(v)))
        dom = domain if rng.random() < 0.97 else "other"
        out.append((dom, ents))
    return out


CONFIG4_N = 1_000_000_000


class Resolve4:
    """The rl_resolve_batch of a config-4 batch: domain "bench4" and the four entries of each
    descriptor are ranges of its own prefix bytes ("bench4_a_<v>_b_<v>_c_<v>_d_<v>_")."""

    def __init__(self, blob: np.ndarray, off: np.ndarray):
        n = int(off.shape[0]) - 1
        o = off[:-1].astype(np.int64)
        nd = (off[1:].astype(np.int64) - o - 22)
        self.bytes, self.bytes_len, self.n_desc, self.n_entries = blob, int(off[-1]), n, 4 * n
        self.domain = np.stack([o, np.full(n, 6)], 1).astype(np.uint32).ravel()
        self.entry_first = (4 * np.arange(n + 1)).astype(np.uint32)
        ent = np.zeros((n, 4, 4), np.int64)
        for e in range(4):
            ent[:, e, 0] = o + 7 + 4 * e
            ent[:, e, 1] = 1
            ent[:, e, 2] = o + 9 + 4 * e
            ent[:, e, 3] = 1 if e < 3 else nd
        self.entry = ent.astype(np.uint32).ravel()

    def struct(self):
        import hiprl
        s = hiprl.RlResolveBatch()
        s.n_desc, s.n_entries, s.bytes_len, s.reserved = self.n_desc, self.n_entries, self.bytes_len, 0
        p = lambda a: a.ctypes.data if a.size else None
        s.bytes, s.domain, s.entry_first, s.entry = p(self.bytes), p(self.domain), p(self.entry_first), p(self.entry)
        s.override_rule = None
        return s

    def descriptors(self):
        """[(domain, [(key, value)...])] for config_oracle.Config.get_limit."""
        out = []
        for i in range(self.n_desc):
            ents = []
            for e in range(4):
                ko, kl, vo, vl = (int(x) for x in self.entry[16 * i + 4 * e:16 * i + 4 * e + 4])
                ents.append((bytes(self.bytes[ko:ko + kl]).decode(), bytes(self.bytes[vo:vo + vl]).decode()))
            do, dl = int(self.domain[2 * i]), int(self.domain[2 * i + 1])
            out.append((bytes(self.bytes[do:do + dl]).decode(), ents))
        return out


def config4_batch(b: int, d: int = 1_000_000, N: int = CONFIG4_N, s: float = 1.1, seed: int = 4,
                  t0: int = 1_700_000_000, batches_per_s: int = 1, hits_max: int = 1):
    """Config 4 (1e9 keys, nested 4-entry descriptors resolved by the config4_yaml tree): Zipf(s)
    ranks through the permutation; key k's entries are a = k % 10, b = k / 10 % 10,
    c = k / 100 % 10, d = k / 1000, so the tree's key/value nodes (values 0..5) and its key-only
    defaults are both taken. Returns (Batch with the rule ids still to resolve, its Resolve4);
    the same layout as tools/gen/workload_gen.hip's mode 3."""
    from hiprl import NIL_RULE
    rank = Zipf(N, s).sample(seed, b, d) - 1
    kv = permute(rank, N)
    ten = np.uint64(10)
    blob, off = prefix_blob([b"bench4_a_", kv % ten, b"_b_", kv // ten % ten, b"_c_", kv // np.uint64(100) % ten,
                             b"_d_", kv // np.uint64(1000), b"_"])
    if hits_max > 1:
        h = (splitmix64(np.uint64(seed) * np.uint64(1 << 40) + np.uint64(b) * np.uint64(1 << 24)
                        + np.arange(d, dtype=np.uint64)) % np.uint64(hits_max) + np.uint64(1)).astype(np.uint32)
    else:
        h = np.ones(d, np.uint32)
    batch = Batch(blob, off, np.full(d, NIL_RULE, np.uint32), np.arange(d, dtype=np.uint32),
                  np.full(d, t0 + b // batches_per_s, np.int64), h)
    return batch, Resolve4(blob, off)


# ---------------------------------------------------------------------------------------
# Config 5: a sustained stream over simulated seconds (window rollover / expiry, variable
# hits_addend h ~ U{1..8}, near-limit ratio 0.8), mixed SECOND / MINUTE / HOUR rules.
# ---------------------------------------------------------------------------------------
CONFIG5_RULES = [(20, SECOND), (400, MINUTE), (9000, HOUR)]


def config5_batch(b: int, d: int, N: int, batches_per_s: int = 1, s: float = 1.1, seed: int = 5,
                  t0: int = 1_700_000_000 - 37) -> Batch:
    """Batch b of config 5: Zipf(1.1) keys over N, rule by rank % 3, 1 descriptor per
    request, h ~ U{1..8} per request, now = t0 + b // batches_per_s (t0 is chosen so the
    stream crosses minute and hour boundaries early)."""
    rank = Zipf(N, s).sample(seed, b, d) - 1
    key = permute(rank, N)
    blob, off = prefix_blob([b"c5_k_", key, b"_"])
    u = splitmix64(np.uint64(seed) * np.uint64(1 << 40) + np.uint64(1 << 32) + np.uint64(b) * np.uint64(1 << 24)
                   + np.arange(d, dtype=np.uint64))
    h = (u % np.uint64(8) + np.uint64(1)).astype(np.uint32)
    return Batch(blob, off, (rank % 3).astype(np.uint32), np.arange(d, dtype=np.uint32),
                 np.full(d, t0 + b // batches_per_s, np.int64), h)

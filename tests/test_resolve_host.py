"""The device GetLimit walk (rl_resolve.hip resolve_one, the code k_resolve runs per
descriptor) executed on the host through tests/cshim/librl_resolve_shim.so, against the config
oracle (oracle/config_oracle.py, GetLimit config_impl.go:274-323, pinned by
tests/test_config_golden.py). CPU only: it covers the register path (strings up to 32 bytes in
whole-dword loads), the byte path (long names, strings whose last dword passes the blob's end,
a blob that is not 4-B aligned) and the bounds checks, on the same source the GPU runs."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

import config_oracle
import hiprl
import rl_config
import workload
from test_config_golden import BASIC, files

SHIM = Path(__file__).resolve().parent / "cshim" / "librl_resolve_shim.so"


@pytest.fixture(scope="module")
def shim():
    if not SHIM.exists():
        subprocess.run(["make", "-C", str(SHIM.parent), SHIM.name], check=True, capture_output=True)
    lib = C.CDLL(str(SHIM))
    lib.rls_resolve.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(hiprl.RlResolveBatch),
                                C.c_void_p]
    lib.rls_resolve.restype = C.c_int
    return lib


def resolve(lib, cfg, rb, shift=0):
    """Rule ids of a ResolveBatch; shift > 0 places the bytes that many bytes past a 16-B
    boundary (offsets unchanged), so the walk sees a blob that is not 4-B aligned."""
    nodes, names = cfg.tree_arrays()
    nodes = np.ascontiguousarray(nodes, np.uint32)
    nb = np.frombuffer(names or b"\0", np.uint8)
    s = rb.struct()
    if shift:
        raw = np.zeros(rb.bytes.size + 32, np.uint8)
        base = (-raw.ctypes.data) % 16 + shift
        raw[base:base + rb.bytes.size] = rb.bytes
        s.bytes = raw.ctypes.data + base
        keep = raw  # noqa: F841 (alive during the call)
    out = np.zeros(max(1, rb.n_desc), np.uint32)
    rc = lib.rls_resolve(nodes.ctypes.data, nodes.shape[0], nb.ctypes.data, len(names), C.byref(s), out.ctypes.data)
    assert rc == 0
    return out[:rb.n_desc]


def _rule_tuple(cfg, rid):
    if rid == hiprl.NIL_RULE:
        return None
    r = cfg.rules[int(rid)]
    return (r.full_key, r.requests_per_unit, r.unit)


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_basic_config(shim, shift):
    """TestBasicConfig's lookups (config_test.go:24-149); the batch's last string ends past the
    blob's last whole dword (the byte path), and shifted blobs take the byte path throughout."""
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    rb = rl_config.ResolveBatch([(d, e, None) for d, e, _ in BASIC])
    got = resolve(shim, cfg, rb, shift)
    assert [_rule_tuple(cfg, r) for r in got] == [w for _, _, w in BASIC]


def test_override(shim):
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    e1 = [("key1", "value1"), ("subkey1", "something")]
    ov = cfg.override_rule("test-domain", e1, 10, 4)
    got = resolve(shim, cfg, rl_config.ResolveBatch([("test-domain", e1, ov), ("foo_domain", [], ov),
                                                       ("test-domain", e1, None)]))
    assert int(got[0]) == ov and got[1] == hiprl.NIL_RULE
    assert _rule_tuple(cfg, got[2]) == ("test-domain.key1_value1.subkey1", 5, 1)


@pytest.mark.parametrize("seed", [4, 5, 6])
def test_config4_tree_against_oracle(shim, seed):
    """A config-4 tree (4 levels, key/value nodes and defaults) and 4000 descriptors that hit
    values, fall back to defaults, use a foreign key or an unknown domain."""
    y = workload.config4_yaml(seed)
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    orc = config_oracle.Config([("c4.yaml", y)])
    descs = workload.config4_descriptors(seed, 4000)
    got = resolve(shim, cfg, rl_config.ResolveBatch([(d, e, None) for d, e in descs]))
    for (d, e), r in zip(descs, got):
        w = orc.get_limit(d, e)
        have = None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
        assert have == (None if w is None else (w.requests_per_unit, w.unit)), (d, e)


def test_long_and_empty_names(shim):
    """Names past the 32 bytes a node holds inline and key "_" value past 32 bytes (the byte
    path), an empty value, and names that share a prefix with a longer one."""
    long_k, long_v = "k" * 30, "v" * 40
    y = (
        "domain: dlong\n"
        "descriptors:\n"
        f"  - key: {long_k}\n"
        f"    value: {long_v}\n"
        "    rate_limit: {unit: second, requests_per_unit: 3}\n"
        f"  - key: {long_k}\n"
        "    rate_limit: {unit: minute, requests_per_unit: 4}\n"
        "  - key: ab\n"
        "    value: c\n"
        "    rate_limit: {unit: hour, requests_per_unit: 5}\n"
        "  - key: a\n"
        "    value: b_c\n"
        "    rate_limit: {unit: day, requests_per_unit: 6}\n"
        "  - key: e\n"
        "    rate_limit: {unit: day, requests_per_unit: 7}\n"
    )
    cfg = rl_config.RateLimitConfig([("l.yaml", y)])
    orc = config_oracle.Config([("l.yaml", y)])
    descs = [("dlong", [(long_k, long_v)]), ("dlong", [(long_k, "x")]), ("dlong", [("ab", "c")]),
             ("dlong", [("a", "b_c")]), ("dlong", [("a", "b")]), ("dlong", [("e", "")]), ("dlong", [("e", "z" * 33)]),
             ("dlong", [(long_k[:-1], long_v)]), ("dlon", [("e", "1")])]
    got = resolve(shim, cfg, rl_config.ResolveBatch([(d, e, None) for d, e in descs]))
    for (d, e), r in zip(descs, got):
        w = orc.get_limit(d, e)
        have = None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
        assert have == (None if w is None else (w.requests_per_unit, w.unit)), (d, e)


def test_strings_outside_bytes_resolve_nil(shim):
    """rl_resolve_device does not refuse a batch (the host form does): a descriptor whose
    domain or entry string lies past bytes_len, or whose entry range passes n_entries,
    resolves to nil and the walk reads nothing outside the arrays."""
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    rb = rl_config.ResolveBatch([("test-domain", [("key3", "foo")], None)] * 3)
    rb.domain = rb.domain.copy()
    rb.entry = rb.entry.copy()
    rb.entry_first = rb.entry_first.copy()
    rb.domain[2 * 0 + 1] = rb.bytes_len + 1       # descriptor 0: domain past the end
    rb.entry[4 * 1 + 2] = rb.bytes_len            # descriptor 1: value offset at the end, length 3
    rb.entry_first[3] = rb.n_entries + 5          # descriptor 2: entries past n_entries
    got = resolve(shim, cfg, rb)
    assert list(got) == [hiprl.NIL_RULE] * 3


# ---- k_resolve's two passes: the level-pipelined walk, then the exact walk for what it leaves ----
def _resolve2(lib, cfg, rb, mode=0, pad=0):
    """(rules, which descriptors the exact walk decided); pad: zero bytes after the blob, so no
    string's load window passes its end."""
    lib.rls_resolve2.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(hiprl.RlResolveBatch),
                                 C.c_void_p, C.c_void_p, C.c_int]
    lib.rls_resolve2.restype = C.c_int
    nodes, names = cfg.tree_arrays()
    nodes = np.ascontiguousarray(nodes, np.uint32)
    nb = np.frombuffer(names or b"\0", np.uint8)
    s = rb.struct()
    raw = np.concatenate([rb.bytes, np.zeros(pad, np.uint8)])
    if pad:
        s.bytes, s.bytes_len = raw.ctypes.data, s.bytes_len + pad
    out = np.zeros(max(1, rb.n_desc), np.uint32)
    ex = np.zeros(max(1, rb.n_desc), np.uint8)
    rc = lib.rls_resolve2(nodes.ctypes.data, nodes.shape[0], nb.ctypes.data, len(names), C.byref(s), out.ctypes.data,
                          ex.ctypes.data, mode)
    assert rc == 0
    return out[:rb.n_desc], ex[:rb.n_desc].astype(bool)


def _colliding(lib, parent, make, count=400_000, fn="rls_tree_hash"):
    """Two distinct names make(i), make(j) with equal edge hash under parent (a birthday search
    over the device's 32-bit edge hash: the exact walk's tree_hash over tree ids, or with
    fn="rls_fast_hash" the first pass's fast_hash over its breadth-first ids)."""
    f = getattr(lib, fn)
    f.argtypes = [C.c_uint32, C.c_char_p, C.c_uint32]
    f.restype = C.c_uint32
    seen = {}
    for i in range(count):
        n = make(i).encode()
        h = f(parent, n, len(n))
        if h in seen:
            return seen[h], i
        seen[h] = i
    raise AssertionError("no 32-bit collision found")


def _mix(k):
    """A name part whose every dword varies with k (the fold is a bijection of the last word, so
    names differing only there never collide)."""
    return format((k * 0x9E3779B97F4A7C15) % (1 << 64), "x")[:6] + str(k)


@pytest.mark.parametrize("seed", [4, 7])
def test_config4_first_pass_decides_and_agrees(shim, seed):
    """On a config-4 tree the level-pipelined pass decides (nearly) every descriptor itself, and
    both passes together give exactly the exact walk's and the oracle's answers."""
    y = workload.config4_yaml(seed)
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    orc = config_oracle.Config([("c4.yaml", y)])
    descs = workload.config4_descriptors(seed, 3000)
    rb = rl_config.ResolveBatch([(d, e, None) for d, e in descs])
    got, ex = _resolve2(shim, cfg, rb)
    exact, _ = _resolve2(shim, cfg, rb, mode=1)
    assert np.array_equal(got, exact)
    # (strings whose 20-B load window passes the blob end take the exact walk: this batch dedupes its
    # strings into a small blob, so a few percent of lookups sit there)
    assert ex.mean() < 0.05, ex.mean()
    for (d, e), r in zip(descs, got):
        w = orc.get_limit(d, e)
        have = None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
        assert have == (None if w is None else (w.requests_per_unit, w.unit)), (d, e)


def _fast_id(lib, cfg, node):
    lib.rls_fast_id.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32]
    lib.rls_fast_id.restype = C.c_uint32
    nodes, names = cfg.tree_arrays()
    nodes = np.ascontiguousarray(nodes, np.uint32)
    nb = np.frombuffer(names or b"\0", np.uint8)
    return lib.rls_fast_id(nodes.ctypes.data, nodes.shape[0], nb.ctypes.data, len(names), node)


@pytest.mark.parametrize("walk", ["fast", "exact"])
def test_edge_hash_collisions_take_the_exact_walk(shim, walk):
    """Sibling names whose 32-bit edge hashes collide. fast: under the first pass's hash, so the
    domain keeps its children in the fast edge table; the first pass takes a probe round's first
    hash match unconfirmed, finds the other name when it confirms the node, and leaves the
    descriptor to the exact walk. exact: under the exact walk's hash, so its own probe meets the
    collision. Either way the answers equal the oracle's (key/value nodes, key-only nodes, a
    colliding name absent from the tree, a collision one level down)."""
    probe = rl_config.RateLimitConfig([("p.yaml", "domain: dc\ndescriptors:\n  - key: a\n    value: x\n")])
    nodes, _ = probe.tree_arrays()
    dom = int(np.nonzero(nodes[:, 0] == 0xFFFFFFFF)[0][0])
    fn = "rls_fast_hash" if walk == "fast" else "rls_tree_hash"
    par = _fast_id(shim, probe, dom) if walk == "fast" else dom
    ci, cj = _colliding(shim, par, lambda k: f"a_{_mix(k)}", fn=fn)
    cp, cq = _colliding(shim, par, lambda k: f"k{_mix(k)}", fn=fn)
    i, j, p, q = _mix(ci), _mix(cj), _mix(cp), _mix(cq)
    y = (
        "domain: dc\n"
        "descriptors:\n"
        f"  - key: a\n    value: \"{i}\"\n    rate_limit: {{unit: second, requests_per_unit: 3}}\n"
        f"    descriptors:\n      - key: b\n        rate_limit: {{unit: day, requests_per_unit: 9}}\n"
        f"  - key: a\n    value: \"{j}\"\n    rate_limit: {{unit: minute, requests_per_unit: 4}}\n"
        "  - key: a\n    rate_limit: {unit: hour, requests_per_unit: 5}\n"
        f"  - key: k{p}\n    rate_limit: {{unit: day, requests_per_unit: 6}}\n"
        f"  - key: k{q}\n    rate_limit: {{unit: second, requests_per_unit: 7}}\n"
    )
    y2 = (
        "domain: dd\n"
        "descriptors:\n"
        f"  - key: a\n    value: \"{i}\"\n    rate_limit: {{unit: second, requests_per_unit: 8}}\n"
        "  - key: a\n    rate_limit: {unit: hour, requests_per_unit: 2}\n"
    )
    files_ = [("c.yaml", y), ("d.yaml", y2)]
    cfg = rl_config.RateLimitConfig(files_)
    orc = config_oracle.Config(files_)
    nodes2, _ = cfg.tree_arrays()
    assert int(np.nonzero(nodes2[:, 0] == 0xFFFFFFFF)[0][0]) == dom  # the hashes were searched under this parent
    assert walk != "fast" or _fast_id(shim, cfg, dom) == par
    descs = [("dc", [("a", str(i))]), ("dc", [("a", str(j))]), ("dc", [("a", "nope")]), ("dc", [(f"k{p}", "v")]),
             ("dc", [(f"k{q}", "v")]), ("dc", [("a", str(i)), ("b", "z")]), ("dc", [("a", str(j)), ("b", "z")]),
             ("dd", [("a", str(j))]), ("dd", [("a", str(i))]), ("dc", [(f"k{q}", "v"), ("b", "z")])]
    got, ex = _resolve2(shim, cfg, rl_config.ResolveBatch([(d, e, None) for d, e in descs]), pad=32)
    exact, _ = _resolve2(shim, cfg, rl_config.ResolveBatch([(d, e, None) for d, e in descs]), mode=1)
    assert np.array_equal(got, exact)
    if walk == "fast":  # a colliding lookup that met the other name first went to the exact walk
        assert ex.any()
    for (d, e), r in zip(descs, got):
        w = orc.get_limit(d, e)
        have = None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
        assert have == (None if w is None else (w.requests_per_unit, w.unit)), (d, e)


def _wide_yaml():
    """A domain with 20 key/value children (more than a fast node holds inline: its children go
    to the fast edge table), a node with exactly 8 children (inline), nested levels under both."""
    lines = ["domain: wide", "descriptors:"]
    for v in range(20):
        lines += [f"  - key: k", f"    value: \"v{v}\"", f"    rate_limit: {{unit: second, requests_per_unit: {v + 1}}}"]
        if v % 5 == 0:
            lines += ["    descriptors:"]
            for c in range(7):
                lines += [f"      - key: s", f"        value: \"{c}\"",
                          f"        rate_limit: {{unit: minute, requests_per_unit: {100 + 10 * v + c}}}"]
            lines += ["      - key: s", "        rate_limit: {unit: hour, requests_per_unit: 7}"]
    lines += ["  - key: k", "    rate_limit: {unit: day, requests_per_unit: 999}"]
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("layout,sep", [("prefix", "_"), ("prefix", ":"), ("dedup", "_")])
def test_fast_tree_layouts_and_overflow(shim, layout, sep):
    """The first pass over its breadth-first tree: a domain whose 20 children live in the fast
    edge table, a node with 8 inline children, misses at both; descriptors laid out as cache-key
    prefixes (key "_" value joined: one load window per entry), the same with another separator
    (the walk must not take key ":" value for key "_" value: it leaves them to the exact walk), and
    deduplicated strings. Answers equal the exact walk's and the oracle's; with the key format's
    own separator the first pass decides everything."""
    y = _wide_yaml()
    cfg = rl_config.RateLimitConfig([("w.yaml", y)])
    orc = config_oracle.Config([("w.yaml", y)])
    rng = np.random.default_rng(7)
    descs = []
    for _ in range(3000):
        ents = [("k", f"v{int(rng.integers(0, 24))}")]
        if rng.random() < 0.7:
            ents.append(("s", str(int(rng.integers(0, 10)))))
        if rng.random() < 0.1:
            ents.append(("t", "x"))
        descs.append(("wide" if rng.random() < 0.97 else "narrow", ents))
    rb = rl_config.ResolveBatch([(d, e, None) for d, e in descs], layout=layout, sep=sep)
    got, ex = _resolve2(shim, cfg, rb, pad=32)
    exact, _ = _resolve2(shim, cfg, rb, mode=1)
    assert np.array_equal(got, exact)
    for (d, e), r in zip(descs, got):
        w = orc.get_limit(d, e)
        have = None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
        assert have == (None if w is None else (w.requests_per_unit, w.unit)), (d, e)
    if sep == "_":
        assert not ex.any()
    else:  # a joined-looking entry with another separator: left to the exact walk, never misread
        assert ex.mean() > 0.5

"""Device GetLimit (rl_load_tree / rl_resolve) against the config oracle, and the config-4
and config-5 shaped streams end to end (resolve on the device -> decide on the device)
against the decision oracle. Runs through the C ABI on an MI355X.

Oracles: oracle/config_oracle.py (GetLimit, config_impl.go:274-323, pinned by
tests/test_config_golden.py) and oracle/rl_oracle.cpp (DoLimit, pinned by
tests/test_oracle_golden.py).
"""
from pathlib import Path

import numpy as np
import pytest

import config_oracle
import hiprl
import oracle
import rl_config
import streams
import workload
from test_config_golden import BASIC, files

pytestmark = pytest.mark.gpu

CFG = Path(__file__).resolve().parent / "golden" / "config"


def _limit_tuple(lim):
    return None if lim is None else (lim.full_key, lim.requests_per_unit, lim.unit)


def _rule_tuple(cfg, rid):
    if rid == hiprl.NIL_RULE:
        return None
    r = cfg.rules[int(rid)]
    return (r.full_key, r.requests_per_unit, r.unit)


def test_resolve_basic_config_gpu():
    """TestBasicConfig's lookups (config_test.go:24-149) on the device."""
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    eng = hiprl.Engine()
    cfg.install(eng)
    got = eng.resolve(rl_config.ResolveBatch([(d, e, None) for d, e, _ in BASIC]))
    assert [_rule_tuple(cfg, r) for r in got] == [w for _, _, w in BASIC]


def test_resolve_override_gpu():
    """TestConfigLimitOverride (config_test.go:151-226): an override applies only when the
    domain exists, and its FullKey is domain "." descriptorToKey."""
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    e1 = [("key1", "value1"), ("subkey1", "something")]
    ov = cfg.override_rule("test-domain", e1, 10, 4)
    ov_foo = cfg.override_rule("foo_domain", [], 10, 4)
    eng = hiprl.Engine()
    cfg.install(eng)
    got = eng.resolve(rl_config.ResolveBatch([("test-domain", e1, ov), ("foo_domain", [], ov_foo),
                                              ("test-domain", e1, None)]))
    assert _rule_tuple(cfg, got[0]) == ("test-domain.key1_value1.subkey1_something", 10, 4)
    assert got[1] == hiprl.NIL_RULE
    assert _rule_tuple(cfg, got[2]) == ("test-domain.key1_value1.subkey1", 5, 1)


@pytest.mark.parametrize("seed", [4, 11])
def test_resolve_random_tree_gpu(seed):
    """A seeded 4-level tree (config 4's shape) and 20k descriptors that hit key/value nodes,
    fall back to key-only defaults, stop early, use a foreign key or an unknown domain."""
    y = workload.config4_yaml(seed)
    orc = config_oracle.Config([("c4.yaml", y)])
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    descs = workload.config4_descriptors(seed, 20_000)
    # colliding splits: ("a_0", ...) vs ("a", "0_...") name the same map key only when equal
    descs += [("bench4", [("a_0", "")]), ("bench4", [("a", "")]), ("bench4", [])]
    eng = hiprl.Engine()
    cfg.install(eng)
    got = eng.resolve(rl_config.ResolveBatch([(d, e, None) for d, e in descs]))
    want = [_limit_tuple(orc.get_limit(d, e)) for d, e in descs]
    have = [_rule_tuple(cfg, r) for r in got]
    bad = [i for i, (a, b) in enumerate(zip(have, want)) if a != b]
    assert not bad, f"{len(bad)} differ; first {descs[bad[0]]}: {have[bad[0]]} vs {want[bad[0]]}"
    assert sum(w is not None for w in want) > 2000  # the walk reaches limits at several depths


def test_resolve_empty_and_errors_gpu():
    eng = hiprl.Engine()
    cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
    cfg.install(eng)
    assert eng.resolve(rl_config.ResolveBatch([])).size == 0
    nodes, names = cfg.tree_arrays()
    dup = np.concatenate([nodes, nodes[1:2]])  # a duplicate (parent, name) edge
    with pytest.raises(hiprl.RedisError):
        eng.load_tree(dup, names)
    fwd = nodes.copy()
    fwd[1, 0] = 5  # a parent after its child
    with pytest.raises(hiprl.RedisError):
        eng.load_tree(fwd, names)


@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("local_cache", [False, True])
def test_config4_stream_resolved_on_device_gpu(local_cache, shadow):
    """Config 4's shape end to end at test size: 4-entry descriptors, device GetLimit, then
    device decisions; the oracle gets the oracle's resolution. Several descriptors per
    request, h in 0..8, the local over-limit cache on and off, and (config 4's shadow mode, an
    extension: tests/test_shadow.py) every other rule of the tree in shadow mode."""
    y = workload.config4_yaml(4)
    orc_cfg = config_oracle.Config([("c4.yaml", y)])
    cfg = rl_config.RateLimitConfig([("c4.yaml", y)])
    eng = hiprl.Engine(local_cache=local_cache)
    cfg.install(eng)
    rules = [tuple(r) for r in cfg.rule_table()]
    if shadow:
        rules = [(r[0], r[1], k % 2 == 0) for k, r in enumerate(rules)]
        eng.load_rules(rules)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=local_cache)
    o.load_rules(rules)
    rng = np.random.default_rng(40)
    t = 1_700_000_000
    n_sh = 0
    for batch in range(6):
        descs = workload.config4_descriptors(100 + batch, 6000, values=40)
        rid = eng.resolve(rl_config.ResolveBatch([(d, e, None) for d, e in descs]))
        want = [orc_cfg.get_limit(d, e) for d, e in descs]
        assert [_rule_tuple(cfg, r) for r in rid] == [_limit_tuple(w) for w in want]
        reqs, i = [], 0
        while i < len(descs):
            n = int(rng.integers(1, 5))
            grp = list(range(i, min(i + n, len(descs))))
            reqs.append((descs[grp[0]][0], [descs[j][1] for j in grp], [int(rid[j]) for j in grp],
                         int(rng.integers(0, 9)), t + batch))
            i += n
        b = hiprl.build_batch(reqs)
        st, thr = eng.submit(b)
        ost, othr = o.submit(b)
        streams.assert_same(st, thr, ost, othr, f"config4 batch {batch} shadow={shadow}")
        if shadow:
            n_sh += int(((st["code_flags"] >> 8) & hiprl.FLAG_SHADOW).astype(bool).sum())
    if shadow:
        assert n_sh > 0


@pytest.mark.parametrize("local_cache", [False, True])
def test_config5_sustained_stream_gpu(local_cache):
    """Config 5's shape at test size: 75 simulated seconds (two batches per second) over
    5000 Zipf keys, mixed SECOND/MINUTE/HOUR rules, h ~ U{1..8}: window rollovers and
    expiry for every unit, near-limit and over-limit stats. Bit-exact against the oracle."""
    eng = hiprl.Engine(local_cache=local_cache)
    eng.load_rules(workload.CONFIG5_RULES)
    o = oracle.Oracle(near_limit_ratio=0.8, local_cache=local_cache)
    o.load_rules(workload.CONFIG5_RULES)
    codes = np.zeros(3, np.int64)
    for b in range(150):
        batch = workload.config5_batch(b, 4000, 5000, batches_per_s=2)
        st, thr = eng.submit(batch)
        ost, othr = o.submit(batch)
        streams.assert_same(st, thr, ost, othr, f"config5 batch {b}")
        c = st["code_flags"] & 0xFF
        codes += np.bincount(c, minlength=3)[:3]
        near = int(st["near_limit_delta"].sum())
        assert near >= 0
    assert codes[1] > 0 and codes[2] > 0  # both OK and OVER_LIMIT decisions occur


def test_resolve_long_names_and_shifted_blob_gpu():
    """Names past the 32 bytes the register path holds (the byte path), key "_" value past 32
    bytes, an empty value, names that share a prefix with a longer one; the batch's bytes also
    at 1-3 bytes past a 16-B boundary (rl_resolve_device on device arrays). Against GetLimit."""
    import torch
    long_k, long_v = "k" * 30, "v" * 40
    y = ("domain: dlong\n"
         "descriptors:\n"
         f"  - key: {long_k}\n    value: {long_v}\n    rate_limit: {{unit: second, requests_per_unit: 3}}\n"
         f"  - key: {long_k}\n    rate_limit: {{unit: minute, requests_per_unit: 4}}\n"
         "  - key: ab\n    value: c\n    rate_limit: {unit: hour, requests_per_unit: 5}\n"
         "  - key: a\n    value: b_c\n    rate_limit: {unit: day, requests_per_unit: 6}\n"
         "  - key: e\n    rate_limit: {unit: day, requests_per_unit: 7}\n")
    cfg = rl_config.RateLimitConfig([("l.yaml", y)])
    orc = config_oracle.Config([("l.yaml", y)])
    descs = [("dlong", [(long_k, long_v)]), ("dlong", [(long_k, "x")]), ("dlong", [("ab", "c")]),
             ("dlong", [("a", "b_c")]), ("dlong", [("a", "b")]), ("dlong", [("e", "")]), ("dlong", [("e", "z" * 33)]),
             ("dlong", [(long_k[:-1], long_v)]), ("dlon", [("e", "1")])] * 40
    eng = hiprl.Engine()
    cfg.install(eng)
    rb = rl_config.ResolveBatch([(d, e, None) for d, e in descs])
    want = []
    for d, e in descs:
        w = orc.get_limit(d, e)
        want.append(None if w is None else (w.requests_per_unit, w.unit))
    have = lambda r: None if r == hiprl.NIL_RULE else (cfg.rules[int(r)].requests_per_unit, cfg.rules[int(r)].unit)
    assert [have(r) for r in eng.resolve(rb)] == want
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    for shift in (1, 2, 3):
        raw = torch.zeros(rb.bytes.size + 64, dtype=torch.uint8, device=dev)
        raw[16 + shift:16 + shift + rb.bytes.size] = torch.from_numpy(rb.bytes.copy()).to(dev)
        keep = [t(rb.domain), t(rb.entry_first), t(rb.entry)]
        s = hiprl.RlResolveBatch()
        s.n_desc, s.n_entries, s.bytes_len, s.reserved = rb.n_desc, rb.n_entries, rb.bytes_len, 0
        s.bytes, s.domain, s.entry_first, s.entry = raw.data_ptr() + 16 + shift, keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr()
        s.override_rule = None
        out = torch.zeros(rb.n_desc, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        eng.resolve_device(s, out.data_ptr())
        torch.cuda.synchronize()
        assert [have(r) for r in out.cpu().numpy().view(np.uint32)] == want, shift


@pytest.mark.parametrize("layout,sep", [("prefix", "_"), ("prefix", ":"), ("dedup", "_")])
def test_resolve_fast_tree_layouts_and_overflow_gpu(layout, sep):
    """k_resolve's first pass on the device over its breadth-first tree: a domain whose 20
    children live in the fast edge table, nodes with 8 inline children, misses at both levels;
    the batch laid out as cache-key prefixes (one load window per key "_" value), with another
    separator (left to the exact walk, never misread as key "_" value), and deduplicated
    strings. Against GetLimit (tests/test_resolve_host.py runs the same walk on the host)."""
    from test_resolve_host import _wide_yaml
    y = _wide_yaml()
    cfg = rl_config.RateLimitConfig([("w.yaml", y)])
    orc = config_oracle.Config([("w.yaml", y)])
    rng = np.random.default_rng(17)
    descs = []
    for _ in range(20_000):
        ents = [("k", f"v{int(rng.integers(0, 24))}")]
        if rng.random() < 0.7:
            ents.append(("s", str(int(rng.integers(0, 10)))))
        if rng.random() < 0.1:
            ents.append(("t", "x"))
        descs.append(("wide" if rng.random() < 0.97 else "narrow", ents))
    eng = hiprl.Engine()
    cfg.install(eng)
    got = eng.resolve(rl_config.ResolveBatch([(d, e, None) for d, e in descs], layout=layout, sep=sep))
    want = [_limit_tuple(orc.get_limit(d, e)) for d, e in descs]
    have = [_rule_tuple(cfg, r) for r in got]
    bad = [i for i, (a, b) in enumerate(zip(have, want)) if a != b]
    assert not bad, f"{len(bad)} differ; first {descs[bad[0]]}: {have[bad[0]]} vs {want[bad[0]]}"
    assert sum(w is not None for w in want) > 5_000


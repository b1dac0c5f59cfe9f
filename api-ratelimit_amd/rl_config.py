"""Host side of descriptor-tree resolution: the reference's config loader, flattened for the
device resolver (rl_load_tree / rl_resolve, include/rl_hip.h).

Mirrors src/config/config_impl.go: loadConfig (:218-250) and loadDescriptors (:115-165)
with validateYamlKeys (:170-214), raising RateLimitConfigError with the reference's
messages ("<file>: descriptor has empty key", "... duplicate descriptor composite key
'<k>'", "... invalid rate limit unit '<u>'", ...). Every node with a rate_limit becomes a
rule of the engine's rule table; its FullKey (the stats key prefix, newRateLimitStats
:65-71) stays here. GetLimit itself (:274-323) runs on the device: `RateLimitConfig.resolve`
builds one rl_resolve_batch for a list of (domain, entries, override) descriptors.
"""

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import ctypes as C
import numpy as np
import yaml

import hiprl

UNIT_VALUE = {"UNKNOWN": 0, "SECOND": 1, "MINUTE": 2, "HOUR": 3, "DAY": 4}
VALID_KEYS = frozenset(("domain", "key", "value", "descriptors", "rate_limit", "unit", "requests_per_unit",
                        "sleep_on_throttle", "report_details"))


class RateLimitConfigError(Exception):
    """config.RateLimitConfigError (src/config/config.go); the reference panics with it."""


@dataclass
class Rule:
    full_key: str            # RateLimit.FullKey: stats prefix
    requests_per_unit: int
    unit: int


class RateLimitConfig:
    """Flattened descriptor trees of one or more YAML files (rateLimitConfigImpl)."""

    def __init__(self, files: Sequence[Tuple[str, str]] = ()):
        self.nodes: List[Tuple[int, int, int, int]] = []  # (parent, name_off, name_len, rule)
        self.names = bytearray()
        self.rules: List[Rule] = []
        self.domain_node: Dict[str, int] = {}
        self._children: Dict[int, Dict[str, int]] = {}
        self._overrides: Dict[Tuple[str, int, int], int] = {}
        for name, text in files:
            self.load(name, text)

    # -- loading (host) -----------------------------------------------------------------
    def _node(self, parent: int, name: str, rule: int) -> int:
        b = name.encode()
        self.nodes.append((parent, len(self.names), len(b), rule))
        self.names += b
        return len(self.nodes) - 1

    @staticmethod
    def _validate(file: str, m) -> None:
        for k, v in m.items():
            if not isinstance(k, str):
                raise RateLimitConfigError(f"{file}: config error, key is not of type string: {k}")
            if k not in VALID_KEYS:
                raise RateLimitConfigError(f"{file}: config error, unknown key '{k}'")
            if isinstance(v, list):
                for e in v:
                    if not isinstance(e, dict):
                        raise RateLimitConfigError(
                            f"{file}: config error, yaml file contains list of type other than map: {e}")
                    RateLimitConfig._validate(file, e)
            elif isinstance(v, dict):
                RateLimitConfig._validate(file, v)

    def _descriptors(self, file: str, parent: int, parent_key: str, descs) -> None:
        seen = self._children.setdefault(parent, {})
        for d in descs or []:
            key = str(d.get("key") or "")
            if key == "":
                raise RateLimitConfigError(f"{file}: descriptor has empty key")
            value = str(d.get("value") or "")
            final_key = key + "_" + value if value else key
            new_parent = parent_key + final_key
            if final_key in seen:
                raise RateLimitConfigError(f"{file}: duplicate descriptor composite key '{new_parent}'")
            rule = hiprl.NIL_RULE
            rl = d.get("rate_limit")
            if rl is not None:
                u = UNIT_VALUE.get(str(rl.get("unit") or "").upper(), 0)
                if u == 0:
                    raise RateLimitConfigError(f"{file}: invalid rate limit unit '{rl.get('unit') or ''}'")
                self.rules.append(Rule(new_parent, int(rl.get("requests_per_unit") or 0), u))
                rule = len(self.rules) - 1
            nid = self._node(parent, final_key, rule)
            seen[final_key] = nid
            self._descriptors(file, nid, new_parent + ".", d.get("descriptors"))

    def load(self, file: str, text: str) -> None:
        try:
            m = yaml.safe_load(text)
        except yaml.YAMLError as ex:
            raise RateLimitConfigError(f"{file}: error loading config file: {ex}")
        m = {} if m is None else m
        if not isinstance(m, dict):
            raise RateLimitConfigError(f"{file}: error loading config file: not a map")
        self._validate(file, m)
        domain = str(m.get("domain") or "")
        if domain == "":
            raise RateLimitConfigError(f"{file}: config file cannot have empty domain")
        if domain in self.domain_node:
            raise RateLimitConfigError(f"{file}: duplicate domain '{domain}' in config file")
        nid = self._node(hiprl.TREE_ROOT, domain, hiprl.NIL_RULE)
        self.domain_node[domain] = nid
        self._descriptors(file, nid, domain + ".", m.get("descriptors"))

    def override_rule(self, domain: str, entries, requests_per_unit: int, unit: int) -> int:
        """The rule for a descriptor.Limit override (config_impl.go:286-296): FullKey =
        domain "." descriptorToKey (:252-264); overrides of one key share its stats."""
        key = ".".join(k + ("_" + v if v else "") for k, v in entries)
        full = domain + "." + key
        k = (full, int(requests_per_unit), int(unit))
        if k not in self._overrides:
            self.rules.append(Rule(full, int(requests_per_unit), int(unit)))
            self._overrides[k] = len(self.rules) - 1
        return self._overrides[k]

    def rule_table(self) -> List[Tuple[int, int]]:
        return [(r.requests_per_unit, r.unit) for r in self.rules]

    def tree_arrays(self) -> Tuple[np.ndarray, bytes]:
        return np.array(self.nodes, np.uint32).reshape(-1, 4), bytes(self.names)

    def install(self, engine: "hiprl.Engine") -> None:
        """Load the rule table and the tree into an engine."""
        engine.load_rules(self.rule_table())
        nodes, names = self.tree_arrays()
        engine.load_tree(nodes, names)


class ResolveBatch:
    """One rl_resolve_batch: descriptors [(domain, [(key, value)...], override_rule or None)].

    layout "dedup": each distinct string once in the blob. "prefix": each descriptor's strings
    inside its own cache-key prefix, domain "_" key "_" value "_" ... (the bytes a batch
    submits anyway), so every entry's value follows its key's separator (sep: that separator,
    "_" as the key format has it; tests vary it)."""

    def __init__(self, descs: Sequence[Tuple[str, Sequence[Tuple[str, str]], Optional[int]]], layout: str = "dedup",
                 sep: str = "_"):
        buf = bytearray()
        cache: Dict[str, Tuple[int, int]] = {}

        def put(s: str) -> Tuple[int, int]:
            r = cache.get(s)
            if r is None:
                b = s.encode()
                r = (len(buf), len(b))
                buf.extend(b)
                cache[s] = r
            return r

        def put_here(s: str) -> Tuple[int, int]:
            b = s.encode()
            r = (len(buf), len(b))
            buf.extend(b)
            return r

        if layout not in ("dedup", "prefix"):
            raise ValueError(f"layout {layout!r}")
        dom, first, ent, ov = [], [0], [], []
        for domain, entries, override in descs:
            if layout == "prefix":
                dom.extend(put_here(domain))
                for k, v in entries:
                    buf.extend(b"_")
                    kr = put_here(k)
                    buf.extend(sep.encode())
                    ent.extend(kr + put_here(v))
                buf.extend(b"_")
            else:
                dom.extend(put(domain))
                for k, v in entries:
                    ent.extend(put(k) + put(v))
            first.append(len(ent) // 4)
            ov.append(hiprl.NIL_RULE if override is None else int(override))
        self.bytes = np.frombuffer(bytes(buf) + b"\0" * 16, np.uint8)
        self.bytes_len = len(buf)
        self.domain = np.array(dom, np.uint32)
        self.entry_first = np.array(first, np.uint32)
        self.entry = np.array(ent, np.uint32)
        self.override = np.array(ov, np.uint32)
        self.n_desc = len(descs)
        self.n_entries = len(ent) // 4
        self.has_override = any(o is not None for _, _, o in descs)

    def struct(self) -> "hiprl.RlResolveBatch":
        s = hiprl.RlResolveBatch()
        s.n_desc, s.n_entries, s.bytes_len, s.reserved = self.n_desc, self.n_entries, self.bytes_len, 0
        p = lambda a: a.ctypes.data if a.size else None
        s.bytes, s.domain, s.entry_first, s.entry = p(self.bytes), p(self.domain), p(self.entry_first), p(self.entry)
        s.override_rule = p(self.override) if self.has_override else None
        return s

"""CPU restatement of the reference's descriptor-tree config (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this; it
is the checker for the device resolver (rl_resolve), never part of the product path.

Follows src/config/config_impl.go of kentik/api-ratelimit:
  * loadDescriptors  :115-165  (finalKey = key["_" value], duplicate / empty-key / unit checks)
  * validateYamlKeys :170-214  (validKeys :49-59)
  * loadConfig       :218-250  (empty / duplicate domain)
  * descriptorToKey  :252-264
  * GetLimit         :274-323  (override first, then the key_value -> key fallback walk)
Stat keys: newRateLimitStats :65-71. Parity is pinned by test/config/config_test.go
(tests/test_config_golden.py transcribes its assertions; basic_config.yaml is copied as a
fixture under tests/golden/).
"""

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import yaml

# pb.RateLimitResponse_RateLimit_Unit_value (go-control-plane v0.9.7 rls v3)
UNIT_VALUE = {"UNKNOWN": 0, "SECOND": 1, "MINUTE": 2, "HOUR": 3, "DAY": 4}

VALID_KEYS = {"domain", "key", "value", "descriptors", "rate_limit", "unit", "requests_per_unit",
              "sleep_on_throttle", "report_details"}  # config_impl.go:49-59


class ConfigError(Exception):
    """RateLimitConfigError: "<file name>: <message>" (config_impl.go:107-109)."""


@dataclass
class Limit:
    full_key: str
    requests_per_unit: int
    unit: int


@dataclass
class Node:
    limit: Optional[Limit] = None
    descriptors: Dict[str, "Node"] = field(default_factory=dict)


def _validate(name: str, m) -> None:
    """validateYamlKeys (config_impl.go:170-214)."""
    for k, v in m.items():
        if not isinstance(k, str):
            raise ConfigError(f"{name}: config error, key is not of type string: {k}")
        if k not in VALID_KEYS:
            raise ConfigError(f"{name}: config error, unknown key '{k}'")
        if isinstance(v, list):
            for e in v:
                if not isinstance(e, dict):
                    raise ConfigError(f"{name}: config error, yaml file contains list of type other than map: {e}")
                _validate(name, e)
        elif isinstance(v, dict):
            _validate(name, v)


def _load_descriptors(name: str, node: Node, parent_key: str, descs) -> None:
    """loadDescriptors (config_impl.go:115-165)."""
    for d in descs or []:
        key = d.get("key") or ""
        if key == "":
            raise ConfigError(f"{name}: descriptor has empty key")
        value = d.get("value") or ""
        final_key = key + ("_" + value if value != "" else "")
        new_parent = parent_key + final_key
        if final_key in node.descriptors:
            raise ConfigError(f"{name}: duplicate descriptor composite key '{new_parent}'")
        limit = None
        rl = d.get("rate_limit")
        if rl is not None:
            unit = str(rl.get("unit") or "").upper()
            if UNIT_VALUE.get(unit, 0) == 0:
                raise ConfigError(f"{name}: invalid rate limit unit '{rl.get('unit') or ''}'")
            limit = Limit(new_parent, int(rl.get("requests_per_unit") or 0), UNIT_VALUE[unit])
        child = Node(limit)
        _load_descriptors(name, child, new_parent + ".", d.get("descriptors"))
        node.descriptors[final_key] = child


class Config:
    """rateLimitConfigImpl: domains -> descriptor trees."""

    def __init__(self, files: List[Tuple[str, str]]):
        self.domains: Dict[str, Node] = {}
        for name, text in files:
            self._load(name, text)

    def _load(self, name: str, text: str) -> None:
        """loadConfig (config_impl.go:218-250)."""
        try:
            any_ = yaml.safe_load(text)
        except yaml.YAMLError as ex:
            raise ConfigError(f"{name}: error loading config file: {ex}")
        if any_ is None:
            any_ = {}
        if not isinstance(any_, dict):
            raise ConfigError(f"{name}: error loading config file: not a map")
        _validate(name, any_)
        domain = any_.get("domain") or ""
        if domain == "":
            raise ConfigError(f"{name}: config file cannot have empty domain")
        if domain in self.domains:
            raise ConfigError(f"{name}: duplicate domain '{domain}' in config file")
        root = Node()
        _load_descriptors(name, root, domain + ".", any_.get("descriptors"))
        self.domains[domain] = root

    @staticmethod
    def descriptor_to_key(entries) -> str:
        """descriptorToKey (config_impl.go:252-264)."""
        out = ""
        for k, v in entries:
            if out != "":
                out += "."
            out += k
            if v != "":
                out += "_" + v
        return out

    def get_limit(self, domain: str, entries, override: Optional[Tuple[int, int]] = None) -> Optional[Limit]:
        """GetLimit (config_impl.go:274-323). entries: [(key, value)]; override: (L, unit)."""
        root = self.domains.get(domain)
        if root is None:
            return None
        if override is not None:
            return Limit(domain + "." + self.descriptor_to_key(entries), override[0], override[1])
        rate_limit = None
        m = root.descriptors
        for i, (k, v) in enumerate(entries):
            nxt = m.get(k + "_" + v)
            if nxt is None:
                nxt = m.get(k)
            if nxt is not None and nxt.limit is not None and i == len(entries) - 1:
                rate_limit = nxt.limit
            if nxt is not None and len(nxt.descriptors) > 0:
                m = nxt.descriptors
            else:
                break
        return rate_limit

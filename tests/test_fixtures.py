"""CPU checks of generated fixtures (no GPU)."""
import inspect
import json
from pathlib import Path

import hiprl
import oracle

GOLDEN = Path(__file__).parent / "golden"


def test_collision_fixture_collides():
    """collisions.json keys agree on exactly the fingerprint bits the fixture claims."""
    c = json.loads((GOLDEN / "collisions.json").read_text())
    assert c["seed"] == inspect.signature(hiprl.Engine).parameters["hash_seed"].default
    for name, shift in (("g35", 29), ("g43", 21)):
        a, b = c[name]
        ha, la = oracle.fingerprint(hiprl.cache_key_prefix("coll", [("k", a)]), c["now"], c["seed"])
        hb, lb = oracle.fingerprint(hiprl.cache_key_prefix("coll", [("k", b)]), c["now"], c["seed"])
        assert ha >> shift == hb >> shift, name
        assert (ha, la) != (hb, lb), name

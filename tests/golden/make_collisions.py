"""Generate tests/golden/collisions.json: key prefixes whose fingerprints collide on the bits
the v4 pipeline buckets and splits by (rl_kernels_v4.hip), for the engine's default
hash seed. Uses the oracle's fingerprint restatement (pinned bit-exact to the device kernel
by tests/test_gpu_golden.py). Run: python tests/golden/make_collisions.py
  - "g35": two keys equal on fingerprint hi bits 29..63 (grouping bits: regrouped in LDS)
  - "g43": two keys equal on hi bits 21..63 (the regroup bits too: LSD-pipeline fallback)
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "api-ratelimit_amd")]
import oracle  # noqa: E402
import workload  # noqa: E402

SEED = 0x5EE7AB1E5EED   # hiprl.Engine default hash_seed
NOW = 1_700_000_000
UNIT = 1                 # SECOND: window start = NOW


def find(shift, n):
    ids = np.arange(n, dtype=np.uint64)
    blob, off = workload.prefix_blob([b"coll_k_", ids, b"_"])
    hi, _ = oracle.fingerprints(blob, off, NOW, SEED)
    g = hi >> np.uint64(shift)
    order = np.argsort(g, kind="stable")
    gs = g[order]
    dup = np.nonzero(gs[1:] == gs[:-1])[0]
    assert len(dup), f"no collision on {64 - shift} bits among {n} keys"
    a, b = int(order[dup[0]]), int(order[dup[0] + 1])
    return [f"{a}", f"{b}"]


out = {"seed": SEED, "now": NOW, "unit": UNIT, "prefix": "coll_k_<id>_",
       "g35": find(29, 600_000), "g43": find(21, 8_000_000)}
(Path(__file__).parent / "collisions.json").write_text(json.dumps(out, indent=1) + "\n")
print(out)

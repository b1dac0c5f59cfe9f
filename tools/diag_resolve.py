"""Diagnostic: BASIC lookups through rl_resolve_device with the bytes aligned and shifted by
1..3 bytes (the byte path), printed against the expected rules."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "api-ratelimit_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np
import torch
import hiprl
import rl_config
from test_config_golden import BASIC, files

cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
eng = hiprl.Engine(lib_path=sys.argv[1] if len(sys.argv) > 1 else None)
cfg.install(eng)
rb = rl_config.ResolveBatch([(d, e, None) for d, e, _ in BASIC])
dev = torch.device("cuda", 0)
want = [None if w is None else w for _, _, w in BASIC]
def tup(r):
    if r == hiprl.NIL_RULE: return None
    x = cfg.rules[int(r)]; return (x.full_key, x.requests_per_unit, x.unit)
for shift in range(4):
    raw = torch.zeros(rb.bytes.size + 64, dtype=torch.uint8, device=dev)
    raw[16 + shift:16 + shift + rb.bytes.size] = torch.from_numpy(rb.bytes.copy()).to(dev)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    keep = [t(rb.domain), t(rb.entry_first), t(rb.entry)]
    s = hiprl.RlResolveBatch()
    s.n_desc, s.n_entries, s.bytes_len, s.reserved = rb.n_desc, rb.n_entries, rb.bytes_len, 0
    s.bytes, s.domain, s.entry_first, s.entry = raw.data_ptr() + 16 + shift, keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr()
    s.override_rule = None
    out = torch.zeros(rb.n_desc, dtype=torch.int32, device=dev)
    eng.resolve_device(s, out.data_ptr())
    torch.cuda.synchronize()
    got = [tup(r) for r in out.cpu().numpy().view(np.uint32)]
    bad = [k for k in range(len(got)) if got[k] != want[k]]
    print("shift", shift, "mismatches", bad, [got[k] for k in bad])

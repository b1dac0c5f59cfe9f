import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "api-ratelimit_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np, torch, hiprl, rl_config
from test_config_golden import BASIC, files
cfg = rl_config.RateLimitConfig(files("basic_config.yaml"))
eng = hiprl.Engine(lib_path=sys.argv[1])
cfg.install(eng)
rb = rl_config.ResolveBatch([(d, e, None) for d, e, _ in BASIC])
dev = torch.device("cuda", 0)
raw = torch.zeros(rb.bytes.size + 64, dtype=torch.uint8, device=dev)
raw[17:17 + rb.bytes.size] = torch.from_numpy(rb.bytes.copy()).to(dev)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
keep = [t(rb.domain), t(rb.entry_first), t(rb.entry)]
torch.cuda.synchronize()
s = hiprl.RlResolveBatch()
s.n_desc, s.n_entries, s.bytes_len, s.reserved = rb.n_desc, rb.n_entries, rb.bytes_len, 0
s.bytes, s.domain, s.entry_first, s.entry = raw.data_ptr() + 17, keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr()
s.override_rule = None
out = torch.zeros(rb.n_desc, dtype=torch.int32, device=dev)
eng.resolve_device(s, out.data_ptr())
torch.cuda.synchronize()
print([hex(x) for x in out.cpu().numpy().view(np.uint32)])

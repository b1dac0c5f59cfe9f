"""Per-phase timing of k_bgroup MSD workgroups from s_memrealtime stamps (diagnostic build lib_S.so)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
import hiprl  # noqa: E402
import workload  # noqa: E402

lp = ROOT / "tools" / "variants" / "lib_S.so"
eng = hiprl.Engine(log2_slots=(22, 24, 25, 12), max_batch_desc=10**6, max_blob_bytes=40 * 10**6, lib_path=lp)
eng.load_rules(workload.CONFIG3_RULES)
dev = torch.device("cuda", 0)
out = torch.empty(10**6 * 20, dtype=torch.uint8, device=dev)
thr = torch.empty(10**6, dtype=torch.int32, device=dev)
for b in range(4):
    hb = workload.config3_batch(b)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    db = [t(hb.blob), t(hb.off.view(np.int32)), t(hb.rule.view(np.int32)), t(hb.req_of.view(np.int32)), t(hb.now),
          t(hb.hits.view(np.int32))]
    torch.cuda.synchronize()
    eng.submit_device_async(hb.n_desc, hb.n_req, int(hb.off[-1]), [x.data_ptr() for x in db], out.data_ptr(),
                            thr.data_ptr())
    eng.wait()
print("stats", eng.stats())
st = np.zeros((2048, 10), np.uint64)
eng.lib.rl_debug_bg_stamps.argtypes = [C.c_void_p, C.c_uint32]
eng.lib.rl_debug_bg_stamps(st.ctypes.data, 2048)
st = st.astype(np.int64)
m = st[:, 9]
msd = np.nonzero((st[:, 7] > 0) & (m > 0))[0]
t0 = st[st[:, 0] > 0, 0].min()
print("MSD blocks with m>0:", len(msd), " m median/max:", np.median(m[msd]), m[msd].max(),
      " mixed:", int((st[msd, 8] == 1).sum()))
rel = (st[msd, :8] - t0) / 100.0
names = ["start", "bases", "loaded", "radix1", "radix2", "radix3", "mixed", "end"]
for k, nm in enumerate(names):
    print(f"  {nm:8s} {rel[:, k].min():8.2f} {np.median(rel[:, k]):8.2f} {rel[:, k].max():8.2f}")
d = np.diff(rel, axis=1)
print("phase durations (median / max):")
for k in range(7):
    print(f"  {names[k]}->{names[k+1]:8s} {np.median(d[:, k]):8.2f} {d[:, k].max():8.2f}")
allend = (st[st[:, 7] > 0, 7] - t0) / 100.0
print("kernel span (first start -> last end): %.2f us" % allend.max())

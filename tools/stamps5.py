"""Per-phase timing of k4_scan from s_memrealtime stamps (diagnostic build
tools/variants/lib_S4.so, built with -DRL_STAMPS). Thread 0 of each block, last batch.
Phases: entry -> fold (per-tile partials) -> column pass -> prefix pass (wave 0 reaches the
tail) -> tail (MSD: range packing; hot: table claims)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
import hiprl  # noqa: E402
import workload  # noqa: E402

lp = ROOT / "tools" / "variants" / "lib_S4.so"
d = 10**6
eng = hiprl.Engine(log2_slots=(22, 24, 25, 12), max_batch_desc=d, max_blob_bytes=40 * d, lib_path=lp)
eng.load_rules(workload.CONFIG3_RULES)
dev = torch.device("cuda", 0)
out = torch.empty(d * 20, dtype=torch.uint8, device=dev)
thr = torch.empty(d, dtype=torch.int32, device=dev)
for b in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    hb = workload.config3_batch(b, d=d)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    db = [t(hb.blob), t(hb.off.view(np.int32)), t(hb.rule.view(np.int32)), t(hb.req_of.view(np.int32)), t(hb.now),
          t(hb.hits.view(np.int32))]
    torch.cuda.synchronize()
    eng.submit_device_async(hb.n_desc, hb.n_req, int(hb.off[-1]), [x.data_ptr() for x in db], out.data_ptr(),
                            thr.data_ptr())
    eng.wait()
print(eng.stats())
st = np.zeros((4096, 8), np.uint64)
eng.lib.rl_debug_st4.argtypes = [C.c_void_p]
assert eng.lib.rl_debug_st4(st.ctypes.data) == 0
a = st[2048:2048 + 96, :5].astype(np.int64)
t0 = a[:, 0].min()
rel = (a - t0) / 100.0
names = ["entry", "fold", "columns", "prefix", "tail"]
for kind, rows in (("hot", rel[:32]), ("msd", rel[32:])):
    print(f"k4_scan {kind} blocks ({len(rows)}): entry min/max {rows[:,0].min():.1f}/{rows[:,0].max():.1f} us, "
          f"end max {rows[:,4].max():.1f} us")
    dd = np.diff(rows, axis=1)
    for j in range(4):
        print(f"   {names[j]:>8s}->{names[j+1]:<8s} median {np.median(dd[:, j]):6.2f}  max {dd[:, j].max():6.2f}")

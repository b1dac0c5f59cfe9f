"""Per-phase timing of the v3 kernels from s_memrealtime stamps (diagnostic build
tools/variants/lib_S3.so, built with -DRL_STAMPS). Stamps are wave 0 of each block; only
blocks stamped during the last batch (within 10 ms of the newest start) are summarised."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
import hiprl  # noqa: E402
import workload  # noqa: E402

lp = ROOT / "tools" / "variants" / "lib_S3.so"
d = 10**6
eng = hiprl.Engine(log2_slots=(22, 24, 25, 12), max_batch_desc=d, max_blob_bytes=40 * d, lib_path=lp)
eng.load_rules(workload.CONFIG3_RULES)
dev = torch.device("cuda", 0)
out = torch.empty(d * 20, dtype=torch.uint8, device=dev)
thr = torch.empty(d, dtype=torch.int32, device=dev)
for b in range(5):
    hb = workload.config3_batch(b, d=d)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    db = [t(hb.blob), t(hb.off.view(np.int32)), t(hb.rule.view(np.int32)), t(hb.req_of.view(np.int32)), t(hb.now),
          t(hb.hits.view(np.int32))]
    torch.cuda.synchronize()
    eng.submit_device_async(hb.n_desc, hb.n_req, int(hb.off[-1]), [x.data_ptr() for x in db], out.data_ptr(),
                            thr.data_ptr())
    eng.wait()
print(eng.stats())
st = np.zeros((4, 4096, 8), np.uint64)
eng.lib.rl_debug_st3.argtypes = [C.c_void_p]
assert eng.lib.rl_debug_st3(st.ctypes.data) == 0
ntiles = (d + 2047) // 2048
names = {0: ("k3_hist", ntiles, ["start", "hot+zero", "loaded", "sorted", "scanned", "end"]),
         3: ("k3_scan", 8, ["start", "folded", "pass1", "pass2", "claimed"]),
         1: ("k3_place", ntiles, ["start", "loaded", "crossing", "end"]),
         2: ("k3_group", (d + 255) // 256, ["start", "staged", "laid", "scanned", "led", "end"])}
for k, (nm, nb, ph) in names.items():
    a = st[k, :nb, :len(ph)].astype(np.int64)
    newest = a[:, 0].max()
    live = (a[:, 0] > newest - 1_000_000) & (a[:, -1] >= a[:, 0])
    a = a[live]
    if not len(a):
        print(nm, "no stamps")
        continue
    t0 = a[:, 0].min()
    rel = (a - t0) / 100.0
    print(f"== {nm}: {len(a)} blocks, span {rel.max():.1f} us; start min/med/max "
          f"{rel[:, 0].min():.1f}/{np.median(rel[:, 0]):.1f}/{rel[:, 0].max():.1f}")
    dd = np.diff(rel, axis=1)
    for j in range(dd.shape[1]):
        print(f"   {ph[j]:>9s}->{ph[j + 1]:<9s} median {np.median(dd[:, j]):7.2f}  "
              f"p90 {np.percentile(dd[:, j], 90):7.2f}  max {dd[:, j].max():7.2f}")
    if k == 2:
        m = st[2, :nb, 7][live]
        print(f"   records per block: median {np.median(m):.0f} max {m.max()}")

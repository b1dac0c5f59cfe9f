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
for b in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
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
# absolute span of each kernel's stamped blocks (s_memrealtime is chip-global): first stamp to
# last stamp, and the gap from the previous kernel's last stamp
spans = {}
for k, (nm, nb, ph) in names.items():
    cols = [0, 5] if k != 2 else [6, 5]
    a0 = st[k, :nb + (1 if k == 2 else 0), cols[0]].astype(np.int64)
    a1 = st[k, :nb + (1 if k == 2 else 0), :].max(axis=1).astype(np.int64)
    ok = a0 > a0.max() - 1_000_000
    spans[nm] = (a0[ok].min(), a1[ok].max())
prev = None
for nm in ["k3_hist", "k3_scan", "k3_place", "k3_group"]:
    b, e = spans[nm]
    gap = "" if prev is None else f"  gap after previous {(b - prev) / 100:.1f} us"
    print(f"{nm:9s} first..last stamp {(e - b) / 100:6.1f} us{gap}")
    prev = e
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
        # every block (empty ranges included): entry stamp 6, exit stamp 5
        ent = st[2, :nb + 1, 6].astype(np.int64)
        ex = st[2, :nb + 1, 5].astype(np.int64)
        ok = ent > ent.max() - 1_000_000
        e0 = ent[ok].min()
        print(f"   all {ok.sum()} blocks: entry span {(ent[ok].max() - e0) / 100:.1f} us, "
              f"last exit {(ex[ok].max() - e0) / 100:.1f} us; entry of block 0 {(ent[0] - e0) / 100:.1f} us")
        live_all = ok & (st[2, :nb + 1, 7] > 0)
        order = np.argsort(ent[ok])
        print("   entry times (us) of blocks by index decile:",
              [round(float((np.median(ent[i:i + nb // 10][ok[i:i + nb // 10]]) - e0) / 100), 1)
               for i in range(0, nb, nb // 10)])

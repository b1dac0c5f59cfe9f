"""Per-phase timing of k4_group from s_memrealtime stamps (diagnostic build
tools/variants/lib_S4.so, built with -DRL_STAMPS). Stamps are wave 0 of each block, last batch."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "api-ratelimit_amd"))
import hiprl  # noqa: E402
import workload  # noqa: E402

lp = ROOT / "tools" / "variants" / (sys.argv[2] if len(sys.argv) > 2 else "lib_S4.so")
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
st = np.zeros((4096, 8), np.uint64)
eng.lib.rl_debug_st4.argtypes = [C.c_void_p]
assert eng.lib.rl_debug_st4(st.ctypes.data) == 0
nb = 1024
a = st[:nb].astype(np.int64)
t0 = a[:, 0].min()
names = ["entry", "staged", "inserted", "reserved", "laidout", "scanned", "led", "done"]
a = a[:, [0, 2, 1, 6, 7, 3, 4, 5]]
a = a[a[:, 1] > 0]
rel = (a[:, :8] - t0) / 100.0
print(f"k4_group {nb} blocks: entry min/med/max {rel[:,0].min():.1f}/{np.median(rel[:,0]):.1f}/{rel[:,0].max():.1f} us;"
      f" last done {rel[:,7].max():.1f} us")
dd = np.diff(rel, axis=1)
for j in range(dd.shape[1]):
    print(f"   {names[j]:>8s}->{names[j + 1]:<8s} median {np.median(dd[:, j]):7.2f}  p90 {np.percentile(dd[:, j], 90):7.2f}"
          f"  max {dd[:, j].max():7.2f}")
print(f"   busy blocks {len(a)}; done time p50/p90/max {np.median(rel[:, 7]):.1f}/{np.percentile(rel[:, 7], 90):.1f}/{rel[:, 7].max():.1f}")
print(f"   staged time p10/p50/p90 {np.percentile(rel[:, 1], 10):.1f}/{np.median(rel[:, 1]):.1f}/{np.percentile(rel[:, 1], 90):.1f}")
# per-block facts (rows 3072 + block, last batch accumulates over the run: divide by batches)
fx = st[3072:3072 + 1024, :4].astype(np.int64)
nbat = int(sys.argv[1]) if len(sys.argv) > 1 else 5
done = np.full(1024, np.nan)
allrel = (st[:1024, 5].astype(np.int64) - t0) / 100.0
ok = st[:1024, 2] > 0
done[ok] = allrel[ok]
order = np.argsort(-np.nan_to_num(done, nan=-1))
print("slowest blocks: block done_us recs/batch keys/batch ranges/batch splits/batch")
for k in order[:12]:
    print(f"   {k:5d} {done[k]:7.1f} {fx[k,0]/nbat:8.1f} {fx[k,1]/nbat:8.1f} {fx[k,2]/nbat:5.2f} {fx[k,3]/nbat:5.2f}")
sel = ok
print("corr(done, recs) = %.2f, corr(done, keys) = %.2f" % (np.corrcoef(done[sel], fx[sel, 0])[0, 1],
                                                           np.corrcoef(done[sel], fx[sel, 1])[0, 1]))
print("median recs/batch %.1f keys/batch %.1f" % (np.median(fx[sel, 0]) / nbat, np.median(fx[sel, 1]) / nbat))

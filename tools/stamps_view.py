"""Summarise raw k4_group / k4_scan phase stamps saved by `bench.py --lib <RL_STAMPS variant>
--dump-stamps FILE.npy` (rows 0..1023: k4_group blocks, wave 0; rows 2048..: k4_scan blocks)."""
import sys

import numpy as np

st = np.load(sys.argv[1]).astype(np.int64)
a = st[:1024]
a = a[a[:, 2] > 0]
if not len(a):  # no k4_group work in the dumped batch (e.g. it fell back): hist rows only
    a = st[:1]
t0 = a[:, 0].min()
names = ["entry", "staged", "inserted", "reserved", "laidout", "scanned", "led", "done"]
rel = (a[:, [0, 2, 1, 6, 7, 3, 4, 5]] - t0) / 100.0
print(f"k4_group {len(a)} busy blocks; last done {rel[:, 7].max():.1f} us, done p50/p90 "
      f"{np.median(rel[:, 7]):.1f}/{np.percentile(rel[:, 7], 90):.1f}")
dd = np.diff(rel, axis=1)
for j in range(dd.shape[1]):
    print(f"   {names[j]:>8s}->{names[j + 1]:<8s} median {np.median(dd[:, j]):7.2f}  p90 {np.percentile(dd[:, j], 90):7.2f}"
          f"  max {dd[:, j].max():7.2f}")
L = st[4000]
if L[0]:
    print(f"last block: epilogue starts {(L[0] - t0) / 100:.1f} us; reductions+occ+hot finalize {(L[1] - L[0]) / 100:.2f},"
          f" candidates {(L[2] - L[1]) / 100:.2f}, ctl clear {(L[3] - L[2]) / 100:.2f} us; ends {(L[3] - t0) / 100:.1f} us")
s5 = st[2048:2048 + 96]
s5 = s5[s5[:, 0] > 0]
if len(s5):
    print(f"k4_scan: {len(s5)} blocks, entry..end {(s5[:, 0].min() - t0) / 100:.1f}..{(s5[:, 4].max() - t0) / 100:.1f} us (k4_group t0)")
h = st[1024:2048]
h = h[h[:, 7] > 0]
if len(h):
    t0h = h[:, 0].min()
    rel = (h - t0h) / 100.0
    nm = ["entry", "hot table", "descs+hash", "partials", "digit pass 1", "digit pass 2", "scan+starts", "written"]
    if len(sys.argv) > 2 and sys.argv[2] == "fine":  # -DRL_HIST_FINE build
        nm = ["entry", "hot table", "level 1", "level 2", "hash+key", "partials", "sort+scan", "written"]
    print(f"k4_hist {len(h)} tiles; entry spread {rel[:, 0].max():.1f} us, last end {rel[:, 7].max():.1f} us, "
          f"end p50 {np.median(rel[:, 7]):.1f}")
    dd = np.diff(rel, axis=1)
    for j in range(7):
        print(f"   {nm[j]:>12s}->{nm[j + 1]:<12s} median {np.median(dd[:, j]):6.2f}  p90 {np.percentile(dd[:, j], 90):6.2f}"
              f"  max {dd[:, j].max():6.2f}")

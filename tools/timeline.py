"""Pipeline timeline of the last batches of a rocprofv3 --kernel-trace run of
`bench.py --no-kernel-times` (every k4 dispatch at the end of the trace is a timed,
pipelined batch).

usage: timeline.py <kernel_trace.csv> [rows]
Prints the last `rows` k4 dispatches (queue, start, end, duration in us relative to the
first shown) and per-batch averages over the last 40 batches: each kernel's duration, the
gap between a batch's k4_group end and the next batch's k4_scan start, and the k4_hist
overlap with the next k4_group."""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 16
ks = []
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
    name = name.replace("void ", "").strip()
    if name.startswith("k4_") or name == "k_resolve":  # (config 4: the resolve of each batch too)
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q))
ks.sort()
show = ks[-n_show:]
t0 = show[0][0]
print(f"{'kernel':10s} {'queue':>6s} {'start':>9s} {'end':>9s} {'dur':>7s}")
for s, e, n, q in show:
    print(f"{n:10s} {q:>6s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}")
by = {n: [(s, e) for s, e, m, _ in ks if m == n] for n in ("k4_hist", "k4_scan", "k4_place", "k4_group")}
B = 40
g, sc, pl, hi = (np.array(by[n][-B:], dtype=np.float64) / 1e3 for n in ("k4_group", "k4_scan", "k4_place", "k4_hist"))
print(f"last {B} batches, us: " + ", ".join(f"{n} {np.mean(x[:, 1] - x[:, 0]):.1f}"
                                           for n, x in (("hist", hi), ("scan", sc), ("place", pl), ("group", g))))
print(f"  step (group end to group end) {np.mean(np.diff(g[:, 1])):.1f}")
print(f"  group end -> next scan start {np.mean(sc[1:, 0] - g[:-1, 1]):.1f}")
print(f"  scan end -> place start {np.mean(pl[:, 0] - sc[:, 1]):.1f};  place end -> group start {np.mean(g[:, 0] - pl[:, 1]):.1f}")
# hist of batch k+1 relative to batch k's scan (the last B hists belong to batches one ahead)
print(f"  hist start - scan start (same step) {np.mean(hi[-B + 1:, 0] - sc[-B:-1, 0]):.1f}; "
      f"hist end - group start {np.mean(hi[-B + 1:, 1] - g[-B:-1, 0]):.1f}")
# slot reuse: batch k's k4_hist writes the device slot of batch k-2, so it must start after
# batch k-2's k4_group ended (the front stream waits for that batch's completion event)
gap2 = hi[2:, 0] - g[:-2, 1]
print(f"  hist(k) start - group(k-2) end: min {gap2.min():.1f} (must be >= 0), mean {gap2.mean():.1f}")

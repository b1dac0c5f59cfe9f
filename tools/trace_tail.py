"""Every dispatch (any kernel) at the end of a rocprofv3 --kernel-trace csv, with queue, start,
end and duration relative to the first one shown, then per-kernel mean durations over the
last `rows` dispatches: the routed step's timeline (bench.py --force-routed).

usage: trace_tail.py <kernel_trace.csv> [rows]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ks = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
    name = name.split("::")[-1] if "<" not in name else name[name.rfind("::", 0, name.find("<")) + 2:]
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:40], q))
ks.sort()
show = ks[-n_show:]
t0 = show[0][0]
print(f"{'kernel':40s} {'queue':>6s} {'start':>9s} {'end':>9s} {'dur':>7s}")
for s, e, n, q in show:
    print(f"{n:40s} {q:>6s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}")
tail = ks[-max(n_show, 400):]
agg = defaultdict(list)
for s, e, n, _ in tail:
    agg[n].append((e - s) / 1e3)
print(f"\nmean over the last {len(tail)} dispatches ({(tail[-1][1] - tail[0][0]) / 1e3:.1f} us span)")
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"{n:40s} n={len(v):4d} mean={sum(v) / len(v):8.1f} us")

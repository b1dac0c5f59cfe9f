"""Host-path timeline from a rocprofv3 --kernel-trace --memory-copy-trace run (measurement
tooling): the last `rows` kernel dispatches and memory copies merged by start time, with
start, end and duration in us relative to the first shown, and the copy direction and size;
then the mean busy time per batch of the H2D and D2H copies over the shown window.

usage: copy_timeline.py <run_kernel_trace.csv> <run_memory_copy_trace.csv> [rows] [skip]
(skip: leave out the last `skip` events, e.g. to look at an earlier round of the bench)"""
import csv
import sys

kt = list(csv.DictReader(open(sys.argv[1])))
mt = list(csv.DictReader(open(sys.argv[2])))
n_show = int(sys.argv[3]) if len(sys.argv) > 3 else 120
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ev = []
for r in kt:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip().split("::")[-1][:28]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?"), ""))
cols = list(mt[0].keys()) if mt else []
for r in mt:
    d = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
    sz = r.get("Bytes") or r.get("Size") or r.get("Copy_Bytes") or ""
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + d[-24:], r.get("Queue_Id", r.get("Stream_Id", "?")), sz))
ev.sort()
if skip:
    ev = ev[:-skip]
show = ev[-n_show:]
t0 = show[0][0]
print("memory copy columns:", cols)
print(f"{'op':36s} {'q':>4s} {'start':>10s} {'end':>10s} {'dur':>8s} {'bytes':>10s}")
for s, e, n, q, sz in show:
    print(f"{n:36s} {q:>4s} {(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {sz:>10s}")
span = (show[-1][1] - t0) / 1e3
busy = {}
for s, e, n, q, sz in show:
    if n.startswith("COPY"):
        busy[n] = busy.get(n, 0.0) + (e - s) / 1e3
print(f"\nwindow {span:.1f} us; copy busy time by direction (us): " + ", ".join(f"{k}: {v:.1f}" for k, v in busy.items()))

"""Per-kernel durations from a rocprofv3 --kernel-trace run of bench.py (tools/pmc_round.sh).

usage: trace_summary.py <run_kernel_trace.csv> <bench.json> <steps> <out.json>

bench.py times each kernel with HIP events over `steps` extra batches run one at a time
(unoverlapped) after the timed region; those are the last `steps` dispatches of every v4
kernel in the trace. This reports the trace's average over exactly those dispatches next to
the bench's own HIP-event averages from the same run, so the two can be compared."""
import collections
import csv
import json
import sys

trace, bench_json, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
durs = collections.defaultdict(list)
rows = list(csv.DictReader(open(trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()
    if k.startswith("k4_"):
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
bk = (bench.get("roofline") or {}).get("kernels_us_per_batch", {})
res = {"steps": steps, "source_sha": bench["engine"]["source_sha"],
       "definition": "trace_avg_us: mean rocprofv3 kernel-trace duration over the last `steps` dispatches "
                     "(bench.py's unoverlapped kernel-timing batches); bench_event_us: bench.py's HIP-event "
                     "average per batch over the same batches",
       "kernels": {k: {"trace_avg_us": round(sum(v[-steps:]) / len(v[-steps:]), 2), "dispatches": len(v),
                       "bench_event_us": bk.get(k)} for k, v in sorted(durs.items())},
       "bench": {"value": bench["value"], "ms_per_step": bench["ms_per_step"]}}
# Timeline of the last batches of the timed (pipelined) region: every dispatch between them,
# including the runtime's blit kernels (control-block copies), to show overlap and gaps.
grp = [r for r in rows if "k4_group" in r["Kernel_Name"]]
if len(grp) >= 2 * steps + 1:
    t_a = int(grp[-steps - 6]["Start_Timestamp"]) - 40_000
    t_b = int(grp[-steps - 1]["End_Timestamp"])
    sel = [r for r in rows if t_a <= int(r["Start_Timestamp"]) <= t_b]
    t0 = int(sel[0]["Start_Timestamp"])
    lines = ["kernel                       queue     start       end     dur"]
    for r in sel:
        k = r["Kernel_Name"].split("(")[0].split("::")[-1].replace("void ", "").strip()[:26]
        a, b = (int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000
        lines.append(f"{k:26s} {r.get('Queue_Id', r.get('Stream_Id', '?')):>7s} {a:9.1f} {b:9.1f} {b - a:7.1f}")
    g = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in grp[-2 * steps:-steps]]
    res["timed_group_period_us"] = round((g[-1][1] - g[0][1]) / (len(g) - 1) / 1000, 2)
    open(out.replace(".json", "_timeline.txt"), "w").write("\n".join(lines) + "\n")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))

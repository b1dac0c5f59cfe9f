"""Per-kernel means of every collected counter over the last <steps> dispatches of each kernel
(tools/pmc_kernels.sh output), with a few derived ratios.

usage: pmc_kernel_counters.py <pmc dir> <out.json> <steps>"""
import collections
import csv
import glob
import json
import sys

root, out, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    recs = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    for r in recs:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        k = k.split("::")[-1].replace("void ", "").strip()
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, c in sorted(rows.items()):
    m = {n: sum(v[-steps:]) / len(v[-steps:]) for n, v in c.items() if v}
    d = {}
    if m.get("SQ_WAVE_CYCLES"):
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in m:
                d[n + "_frac"] = round(m[n] / m["SQ_WAVE_CYCLES"], 4)
    if m.get("SQ_WAVES") and m.get("SQ_INSTS_VMEM_RD"):
        d["vmem_rd_per_wave"] = round(m["SQ_INSTS_VMEM_RD"] / m["SQ_WAVES"], 2)
    if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None and m["TCC_HIT_sum"] + m["TCC_MISS_sum"]:
        d["l2_hit_rate"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    res[k] = {"dispatches": max(len(v) for v in c.values()), "mean": {n: round(v, 1) for n, v in m.items()}, "derived": d}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k.startswith(("k_resolve", "k4_"))}, indent=1))

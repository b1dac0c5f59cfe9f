"""Per-kernel HBM traffic from rocprofv3 --pmc passes (tools/pmc_round.sh output).

usage: pmc_traffic.py <pmc dir> <out.json> <timed steps> [tag] [bench config]

Only the last <timed steps> dispatches of each kernel are used: the bench's timed region
(prefill and warmup dispatches run at other table fills and are skipped). FETCH_SIZE and
WRITE_SIZE are KiB per dispatch. Per MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE counts half
the bytes of a wide coalesced read, so hbm_bytes_per_launch = 2 x FETCH + WRITE. Random 32-B
slot traffic is calibrated separately on tools/microbench/table_rmw (random 32-B probe reads
and 32-B read-modify-writes of known count on an 8 GiB table): the calibration block reports
counter bytes per operation for those access shapes, so the reader can see how the counters
tally the table's random accesses. The summary carries bench.source_sha(), so bench.py uses
it only for the kernel sources it was measured on."""
import collections
import csv
import glob
import json
import os
import sys

root, out, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
tag = sys.argv[4] if len(sys.argv) > 4 else ""
config = int(sys.argv[5]) if len(sys.argv) > 5 else 3
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import source_sha  # noqa: E402


def kname(r):
    # (k_resolve lives in an anonymous namespace: drop that before cutting at the arguments)
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
    return k.split("::")[-1].replace("void ", "").strip()


def load(pattern, timed=0):
    """kernel -> counter -> [values in dispatch order]. timed > 0: per pass, only the dispatches
    after the k4_group of the batch before the last `timed` ones (the timed region: the LSD
    pipeline's prefill fallbacks and other prefill work drop out, whatever their count)."""
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(pattern):
        recs = list(csv.DictReader(open(f)))
        recs.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        t0 = -1
        if timed:
            g = sorted({int(r.get("Dispatch_Id", 0) or 0) for r in recs if kname(r) == "k4_group"})
            if len(g) > timed:
                t0 = g[-(timed + 1)]
        for r in recs:
            if int(r.get("Dispatch_Id", 0) or 0) > t0:
                rows[kname(r)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


def mean_last(v, n):
    v = v[-n:] if n else v
    return sum(v) / len(v) if v else 0.0


bench_rows = load(f"{root}/p*/run_counter_collection.csv", steps)
# the bench's workload generator (tools/gen/workload_gen.hip) and roofline probe: not the path
NOT_ENGINE = ("k_keys", "k_bytes", "k_bytes4", "k_copy", "k_slot_rmw")
kernels = {}
for k, c in sorted(bench_rows.items()):
    if not k.startswith(("k_", "k4_")) or k in NOT_ENGINE:
        continue
    n = len(c.get("FETCH_SIZE", []))
    f = mean_last(c.get("FETCH_SIZE", []), steps) * 1024
    w = mean_last(c.get("WRITE_SIZE", []), steps) * 1024
    hit, miss = mean_last(c.get("TCC_HIT_sum", []), steps), mean_last(c.get("TCC_MISS_sum", []), steps)
    kernels[k] = {"dispatches_seen": n, "fetch_size_bytes": round(f), "write_size_bytes": round(w),
                  "hbm_bytes_per_launch": round(2 * f + w),
                  "tcc_ea0_atomic": round(mean_last(c.get("TCC_EA0_ATOMIC_sum", []), steps)),
                  "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None}
cal_rows = load(f"{root}/c*/run_counter_collection.csv")
U = 230000
cal = {}
for k, c in cal_rows.items():
    if k not in ("k_probe_read", "k_rmw", "k_copy"):
        continue
    # table_rmw launches each kernel 1 + reps times; every launch touches the same U slots
    f = mean_last(c.get("FETCH_SIZE", []), 0) * 1024
    w = mean_last(c.get("WRITE_SIZE", []), 0) * 1024
    cal[k] = {"fetch_size_bytes_per_op": round(f / U, 2), "write_size_bytes_per_op": round(w / U, 2)}
cal["note"] = ("k_probe_read: one random 16-B load per op inside a 32-B slot; k_rmw: random 32-B slot "
               "load + store per op (two 16-B lanes); U = 230000 ops per launch on 2^28 slots")
res = {"tag": tag, "source_sha": source_sha(), "config": config, "timed_steps": steps,
       "hbm_bytes_per_batch": sum(v["hbm_bytes_per_launch"] for v in kernels.values() if v["dispatches_seen"] >= steps),
       "definition": "hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md gfx950 FETCH_SIZE "
                     "correction), mean over the last timed_steps dispatches of each kernel",
       "kernels": kernels, "calibration_table_rmw": cal}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))

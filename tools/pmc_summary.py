"""Summarise rocprofv3 --pmc CSVs (one dir per pass) per kernel: mean counter value per dispatch."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("rlhip::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(f"{root}/p*/run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("rlhip::", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k in acc:
    c = acc[k]
    d = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else 0
    line = {n: sum(v) / len(v) for n, v in c.items()}
    print(f"== {k}  median {d:.1f} us")
    for n, v in sorted(line.items()):
        print(f"   {n:22s} {v:16.0f}")

"""Per-dispatch durations of each kernel, in dispatch order, bucketed (rocprofv3 --kernel-trace csv of
tools/step_overhead.py): which kernel runs slow in the first steps after start?
Usage: python tools/warm_trace.py <kernel_trace.csv> [bucket]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = defaultdict(list)
for r in rows:
    per[re.split(r"[<(]", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    if len(d) < 2 * bucket:
        continue
    means = [sum(d[i:i + bucket]) / len(d[i:i + bucket]) for i in range(0, min(len(d), 12 * bucket), bucket)]
    print(f"{name:60s} n={len(d):5d} " + " ".join(f"{m:6.1f}" for m in means) + f"  | last {sum(d[-64:]) / 64:6.1f}")

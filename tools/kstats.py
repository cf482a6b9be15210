"""Print a rocprofv3 kernel_stats.csv as per-step milliseconds (usage: kstats.py <csv> [steps])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    n = r["Name"].replace("(anonymous namespace)::", "")[:100]
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:7.1f} calls "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us {float(r['Percentage']):5.1f}%  {n}")
print(f"total {tot / 1e6 / steps:.3f} ms/step")

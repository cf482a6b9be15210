"""Top kernels of a rocprofv3 --stats run: python tools/show_stats.py <output dir> [top]  (reads *kernel_stats.csv)"""
import csv
import glob
import sys

path = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(path, f"total {tot / 1e6:.2f} ms")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.3f}ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f}us "
          f"{float(r['Percentage']):5.1f}% {r['Name'][:120]}")

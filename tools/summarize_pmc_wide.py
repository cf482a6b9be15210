"""Average PMC counter value per dispatch and kernel from tools/pmc_wide.sh output (usage: TAG)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "wide"
acc = defaultdict(lambda: [0.0, 0])
for f in glob.glob(f"gpurun_out/pmcw_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        key = (name, r["Counter_Name"])
        acc[key][0] += float(r["Counter_Value"])
        acc[key][1] += 1
by_kernel = defaultdict(dict)
disp = defaultdict(set)
for (k, c), (v, n) in acc.items():
    by_kernel[k][c] = v
for f in glob.glob(f"gpurun_out/pmcw_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        disp[(name, f)].add(r["Dispatch_Id"])
for k, cs in by_kernel.items():
    nd = max(len(v) for (kk, f), v in disp.items() if kk == k)
    print(k, f"({nd} dispatches per pass)")
    for c in sorted(cs):
        print(f"   {c:28s} {cs[c] / nd:16.0f}")

"""Per-kernel averages of the instruction / stall counters collected by tools/pmc_insts.sh.
Usage: python tools/summarize_pmc.py TAG  -> prints and writes profiles/<TAG>_pmc_insts.csv"""
import csv
import glob
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "gpurun_out", f"pmc_{tag}", "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = next((k for k in ("k_forward", "k_backward", "k_reduce", "k_inverse", "k_pack", "k_hp", "k_dh",
                                  "k_dw1h_reduce", "k_dw1h") if k in name), None)
        if short is None:
            continue
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, d in sorted(acc.items()):
    for c, v in sorted(d.items()):
        rows.append((k, c, sum(v) / len(v)))
w = os.path.join(root, "profiles", f"{tag}_pmc_insts.csv")
with open(w, "w") as f:
    f.write("kernel,counter,avg_per_dispatch\n")
    for k, c, v in rows:
        f.write(f"{k},{c},{v:.1f}\n")
for k, d in sorted(acc.items()):
    waves = sum(d["SQ_WAVES"]) / max(1, len(d["SQ_WAVES"])) if "SQ_WAVES" in d else None
    print(f"== {k} (waves/dispatch {waves})")
    for c, v in sorted(d.items()):
        a = sum(v) / len(v)
        per = f"  per-wave {a / waves:12.1f}" if waves else ""
        print(f"   {c:28s} {a:16.1f}{per}")

"""profiles/pmc_wide.json from tools/pmc_wide.sh output: per wide workload, the chain GEMM kernels' (k_wbr ACT / GRAD)
and the whole coupling stack's matrix-pipe busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x duration x clock),
with durations from the same run's kernel trace. python tools/pmc_wide.py TAG"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_SIMD, CLOCK_GHZ = 1024, 2.4
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()


def main(tag):
    src = os.path.join(root, "gpurun_out", f"pmcw_{tag}")
    out = {}
    for wl in ("fc_large", "lstm_large"):
        st = glob.glob(os.path.join(src, f"trace_{wl}", "**", "*kernel_stats.csv"), recursive=True)
        pc = glob.glob(os.path.join(src, f"pmc_{wl}", "**", "*counter_collection.csv"), recursive=True)
        if not st or not pc:
            continue
        dur = {short(r["Name"]): (float(r["AverageNs"]), int(r["Calls"])) for r in csv.DictReader(open(st[0]))}
        cnt = defaultdict(lambda: defaultdict(float))
        ndisp = defaultdict(set)
        for r in csv.DictReader(open(pc[0])):
            k = short(r.get("Kernel_Name") or r.get("Kernel-Name") or "")
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            ndisp[k].add(r.get("Dispatch_Id") or r.get("Dispatch-Id"))
        res = {}
        tot_busy = tot_ns = 0.0
        for k, c in cnt.items():
            n = max(len(ndisp[k]), 1)
            if k not in dur or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
                continue
            ns = dur[k][0]
            busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / n
            res[k] = {"avg_us": round(ns / 1e3, 2), "mfma_busy_frac": round(busy / (N_SIMD * ns * CLOCK_GHZ), 4),
                      "valu_per_mfma": round(c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 1), 1), 2)}
            if k.startswith(("k_w", "k_gemm", "k_lin", "k_skinny")):
                tot_busy += busy * dur[k][1]
                tot_ns += ns * dur[k][1]
        chain = {k: v for k, v in res.items() if k.startswith("k_wbr")}
        out[wl] = {"chain": chain, "library_kernels_mfma_busy_frac":
                   round(tot_busy / (N_SIMD * tot_ns * CLOCK_GHZ), 4) if tot_ns else None, "kernels": res}
    path = os.path.join(root, "profiles", "pmc_wide.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({w: {"chain": v["chain"], "all": v["library_kernels_mfma_busy_frac"]} for w, v in out.items()},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r04")

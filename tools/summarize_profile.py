"""Turn a tools/profile_round.sh output dir into committed summaries under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats kernel summary (the bench command)
  profiles/<tag>_pmc_traffic.csv    per-kernel HBM bytes per launch from FETCH_SIZE / WRITE_SIZE
  profiles/pmc_traffic.json         {kernel: bytes_per_launch} read by bench.py (roofline.traffic)
  profiles/<tag>_pmc_insts.csv      per-kernel SQ counters per launch (waves, MFMA busy cycles, VALU / MFMA / LDS
                                    instructions, LDS bank conflicts)
  profiles/pmc_insts.json           {kernel: {counter: per_launch}} read by bench.py (roofline.mfma_busy_frac, ...)
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced stream (MI355X_MICROARCH.md §HBM), so traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024."""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", f"prof_{tag}")
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)

stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    print("kernel stats:", stats[0])
for wl in ("resim", "sample", "fc_large"):        # other workloads' --stats runs (tools/round_evidence.sh)
    st2 = glob.glob(os.path.join(src, "trace_" + wl, "**", "*kernel_stats.csv"), recursive=True)
    if st2:
        shutil.copy(st2[0], os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))


def short(name):
    for k in ("k_forward", "k_backward", "k_inverse", "k_red_gx", "k_fold_splitk", "k_fold_finish", "k_pack_fold",
              "k_bwd_tail", "k_adam", "k_clip", "k_pack", "k_hp", "k_resim"):
        if k in name:
            return k
    return None


def per_kernel(counter_glob, counter):
    out = {}
    for f in glob.glob(os.path.join(src, counter_glob, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k and r["Counter_Name"] == counter:
                out.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


INSTS = ("SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
         "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT")
insts = {}
for c in INSTS:
    for k, v in per_kernel("insts", c).items():
        insts.setdefault(k, {})[c] = round(v, 1)
if insts:
    with open(os.path.join(dst, f"{tag}_pmc_insts.csv"), "w") as f:
        f.write("kernel," + ",".join(INSTS) + "\n")
        for k in sorted(insts):
            f.write(k + "," + ",".join(str(insts[k].get(c, "")) for c in INSTS) + "\n")
    with open(os.path.join(dst, "pmc_insts.json"), "w") as f:
        json.dump(insts, f, indent=1)
    print(json.dumps(insts, indent=1))


fetch = per_kernel("fetch", "FETCH_SIZE")
write = per_kernel("write", "WRITE_SIZE")
rows, traffic = [], {}
for k in sorted(set(fetch) | set(write)):
    fb = 2.0 * fetch.get(k, 0.0) * 1024
    wb = write.get(k, 0.0) * 1024
    traffic[k] = round(fb + wb)
    rows.append({"kernel": k, "FETCH_SIZE_KiB": round(fetch.get(k, 0.0), 1), "WRITE_SIZE_KiB": round(write.get(k, 0.0), 1),
                 "hbm_bytes_per_launch": round(fb + wb)})
if rows:
    with open(os.path.join(dst, f"{tag}_pmc_traffic.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
print(json.dumps(rows, indent=1))

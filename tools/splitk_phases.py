"""Phase timing of the folded split-K launch (k_fold_splitk, FC_small B=4096), per workgroup from s_memrealtime
stamps (100 MHz) of an experiment build with BCNF_EXP & 32768: dispatch spread, operand-load round trip, LDS staging,
MFMAs, stores. Runs tools/fold_bench.py first (its last launch is the padded-x fold tail TrainStep uses).
Usage (GPU box): BCNF_AMD_LIB=build_exp/libexp32768.so python tools/splitk_phases.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    sys.argv = [sys.argv[0], "--iters", "20"]
    from tools import fold_bench
    fold_bench.main()
    from bcnf_amd import _native as N
    L = N.lib()
    buf = (ctypes.c_ulonglong * (1024 * 5))()
    if not hasattr(L, "bcnf_debug_splitk") or L.bcnf_debug_splitk(buf):
        print("no split-K stamps (build with BCNF_EXP & 32768)")
        return
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 5).astype(np.int64)
    a = a[a[:, 0] > 0]
    n = len(a)
    t0 = a[:, 0].min()
    us = (a - t0) * 0.01          # 100 MHz ticks -> us
    print(f"workgroups stamped: {n}")
    names = ["start", "loads landed", "LDS staged", "MFMAs done", "stored"]
    for i, nm in enumerate(names):
        v = us[:, i]
        print(f"  {nm:13s} abs us: min {v.min():7.2f}  median {np.median(v):7.2f}  max {v.max():7.2f}")
    d = np.diff(us, axis=1)
    for i in range(4):
        v = d[:, i]
        print(f"  {names[i]:>13s} -> {names[i + 1]:13s}: median {np.median(v):6.2f}  p90 {np.percentile(v, 90):6.2f}"
              f"  max {v.max():6.2f} us")
    order = np.argsort(a[:, 0])
    print("  first 8 starts (us):", np.round(us[order[:8], 0], 2).tolist())
    print("  last 8 starts (us):", np.round(us[order[-8:], 0], 2).tolist())


if __name__ == "__main__":
    main()

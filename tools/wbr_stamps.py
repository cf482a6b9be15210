"""Phase stamps of the wide chain GEMM (tiling W, k_wbr) from a diagnostic build (-DBCNF_PHASE_STAMPS,
tools/exp_variants.sh): runs FC_large forward (+ backward) passes, then reads wave 0 of the first 256 tiles of the
LAST k_wbr launch (the forward's last ACT GEMM, or the backward's last GRAD GEMM) and prints medians / percentiles of
the cycles to: A + band issued, band landed (barrier), K loop done, KS merge done, epilogue stores done; and the clock.
Usage: BCNF_AMD_LIB=build_exp/libstamps.so python tools/wbr_stamps.py [--batch 2048]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def read(L):
    buf = (ctypes.c_ulonglong * (256 * 8))()
    assert L.bcnf_wide_debug_wbr(buf) == 0
    return torch.tensor(list(buf), dtype=torch.float64).view(256, 8)


def report(name, t):
    t = t[t[:, 6] > 0]
    q = lambda col, p: float(torch.quantile(t[:, col], p))            # noqa: E731
    names = ["issued", "band landed", "K loop done", "KS merge", "epilogue done"]
    print(f"{name}: {t.shape[0]} tiles; cycles median (p10 / p90):")
    for i, n in enumerate(names):
        print(f"   {n:14s} {q(i, .5):8.0f}  ({q(i, .1):.0f} / {q(i, .9):.0f})")
    ghz = t[:, 6] / (t[:, 5] * 10.0)
    print(f"   clock {float(ghz.median()):.3f} GHz; wave life {float((t[:, 5] * 10 / 1e3).median()):.2f} us (median)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--workload", default="fc_large")
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    from bench import FC_LARGE, LSTM_LARGE
    torch.manual_seed(0)
    cfg = FC_LARGE if args.workload == "fc_large" else LSTM_LARGE
    m = CondRealNVP_v2.from_config(cfg).cuda().train()
    st = m.fused
    B = args.batch
    y = torch.randn(B, 19, device="cuda")
    h = torch.randn(B, 1360, device="cuda")
    L = N.lib()
    if not hasattr(L, "bcnf_wide_debug_wbr"):
        print("not a diagnostic build")
        return
    L.bcnf_wide_debug_wbr.argtypes = [ctypes.c_void_p]
    for _ in range(3):      # warm (clock)
        z, _, vals, saved = st.launch_nll_forward(y, h, True)
        st.launch_nll_backward(h, z, None, True, saved, want_dy=False, want_dh=True)
    z, _, vals, saved = st.launch_nll_forward(y, h, True)
    torch.cuda.synchronize()
    report("ACT (forward's last chain GEMM)", read(L))
    st.launch_nll_backward(h, z, None, True, saved, want_dy=False, want_dh=True)
    torch.cuda.synchronize()
    report("GRAD (backward's last chain GEMM)", read(L))


if __name__ == "__main__":
    main()

"""Kernel micro-benchmark: times the fused forward / backward / inverse kernels in isolation (HIP events),
FC_small shape, for quick A/B of kernel changes. Usage: python tools/kbench.py [--batch 4096] [--iters 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--train", type=int, default=1)
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bench import FC_SMALL
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL).cuda()
    st = m.fused
    B = args.batch
    y = torch.randn(B, 19, device="cuda")
    h = torch.randn(B, 80, device="cuda")
    dz = torch.randn(B, 19, device="cuda")
    dl = torch.randn(B, device="cuda")
    train = bool(args.train)
    res = {}
    for it in range(args.iters + 3):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        z, ldj, _, saved = st.launch_forward(y, h, train, save=True)
        e[1].record()
        st.launch_backward(h, dz, dl, train, saved, want_dy=False, want_dh=True)
        e[2].record()
        with torch.no_grad():
            st.launch_inverse(z, h)
        e[3].record()
        torch.cuda.synchronize()
        if it >= 3:
            for k, (a, b) in {"fwd+pack": (0, 1), "bwd+reduce": (1, 2), "inverse+pack": (2, 3)}.items():
                res.setdefault(k, []).append(e[a].elapsed_time(e[b]) * 1e3)
    # NLL-fused forward (last-workgroup epilogue) vs plain forward
    for name, fn in (("fwd plain", lambda: st.launch_forward(y, h, train, save=True)),
                     ("fwd nll", lambda: st.launch_nll_forward(y, h, train))):
        for it in range(args.iters + 3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            if it >= 3:
                res.setdefault(name, []).append(a.elapsed_time(b) * 1e3)
    for k, v in res.items():
        v.sort()
        print(f"{k:14s} median {v[len(v)//2]:8.1f} us   min {v[0]:8.1f} us")




def phases():
    """Per-phase cycles of the backward loop, workgroup 0 (diagnostic build: bash tools/exp_variants.sh stamps)."""
    import ctypes
    from bcnf_amd import _native as N
    L = N.lib()
    if not hasattr(L, "bcnf_debug_phases"):
        return
    buf = (ctypes.c_ulonglong * 32)()
    L.bcnf_debug_phases(buf)
    names = ["bwd compute: prologue", "bwd compute: chain", "bwd compute: barrier wait", "-",
             "bwd helper: loop top/barrier", "bwd helper: prep_load issue", "bwd helper: grad jobs",
             "bwd helper: prep_store", "fwd compute: prologue", "fwd compute: chain", "fwd compute: barrier wait", "-",
             "fwd helper: prologue", "fwd helper: prepare", "fwd helper: barrier wait", "-"]
    for i, n in enumerate(names):
        if n != "-":
            print(f"  {n:26s} {buf[i]:10d} cycles")


if __name__ == "__main__":
    main()
    phases()

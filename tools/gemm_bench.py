"""Time the wide-family GEMM tilings (bcnf_wide_gemm_test) against torch.matmul (hipBLASLt) on the FC_large shapes.
Usage (GPU box): python tools/gemm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcnf_amd import _native as N  # noqa: E402


def bench(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    L = N.lib()
    shapes = [(2048, 528, 528), (1024, 528, 528), (2048, 13728, 1360), (2048, 1360, 13728), (528, 528, 2048)]
    tilings = (1, 2, 3, 4, 5, 6, 7)
    if len(sys.argv) > 1 and "x" in sys.argv[1]:      # explicit shapes MxNxK[,MxNxK...] [tilings t,t,...] [layouts]
        shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1].split(",")]
        if len(sys.argv) > 2:
            tilings = tuple(int(t) for t in sys.argv[2].split(","))
    elif len(sys.argv) > 1:
        shapes = shapes[:int(sys.argv[1])]
    layouts = (0, 1, 2) if len(sys.argv) <= 3 else tuple(int(v) for v in sys.argv[3].split(","))
    for (M, Nn, K) in shapes:
        for layout in layouts:
            if layout == 2:
                A = torch.randn(K, M, device=dev)
            else:
                A = torch.randn(M, K, device=dev)
            B = torch.randn(Nn, K, device=dev) if layout == 0 else torch.randn(K, Nn, device=dev)
            C = torch.empty(M, Nn, device=dev)
            st = N.stream_handle(dev)
            res = []
            for t in tilings:
                def f():
                    L.bcnf_wide_gemm_test(layout | (t << 4), M, Nn, K, N.ptr(A), A.shape[1], N.ptr(B), B.shape[1],
                                          N.ptr(C), Nn, st)
                us = bench(f)
                res.append(f"t{t}={us:7.1f}us {2 * M * Nn * K / us / 1e6:6.1f}TF")
            if layout == 0:
                ref = bench(lambda: torch.matmul(A, B.t(), out=C))
            elif layout == 1:
                ref = bench(lambda: torch.matmul(A, B, out=C))
            else:
                ref = bench(lambda: torch.matmul(A.t(), B, out=C))
            res.append(f"torch={ref:7.1f}us {2 * M * Nn * K / ref / 1e6:6.1f}TF")
            print(f"M={M:6d} N={Nn:6d} K={K:6d} layout={layout}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()

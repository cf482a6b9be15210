"""Tiling W (LDS-resident B band, t10) vs tiling C (t6) on K-contiguous x K-contiguous shapes: max error vs an fp64
matmul, and time per launch (back-to-back launches, HIP events).
Usage (GPU box): python tools/gemm_rd.py [MxNxK,...] [tilings t,t,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcnf_amd import _native as N  # noqa: E402


def bench(fn, iters=20, reps=10):
    """Device time per launch: `iters` launches captured in one HIP graph (no host launch cost), replayed."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(iters):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * reps)


def main():
    dev = torch.device("cuda")
    L = N.lib()
    shapes = [(2048, 528, 528), (1024, 528, 528), (2048, 526, 528), (37, 528, 528), (300, 100, 44)]
    tilings = (6, 10)
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1].split(",")]
    if len(sys.argv) > 2:
        tilings = tuple(int(t) for t in sys.argv[2].split(","))
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, Nn, K) in shapes:
        A = torch.randn(M, K, device=dev, generator=g)
        B = torch.randn(Nn, K, device=dev, generator=g)
        ref = (A.double() @ B.double().t())
        scale = (A.double().abs() @ B.double().abs().t()).max().item()
        res = []
        for t in tilings:
            C = torch.full((M, Nn), float("nan"), device=dev)

            pa, pb, pc = N.ptr(A), N.ptr(B), N.ptr(C)

            def f():
                rc = L.bcnf_wide_gemm_test(0 | (t << 4), M, Nn, K, pa, K, pb, K, pc, Nn,
                                           N.stream_handle(dev))
                assert rc == 0, rc
            f()
            torch.cuda.synchronize()
            err = (C.double() - ref).abs().max().item() / scale
            us = bench(f)
            res.append(f"t{t}={us:6.1f}us {2 * M * Nn * K / us / 1e6:5.1f}TF err={err:.1e}")
        print(f"M={M:5d} N={Nn:4d} K={K:4d}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()

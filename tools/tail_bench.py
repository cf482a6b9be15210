"""Backward-tail role timing (FC_small): the full tail (dh + slab reduce + W1 condition split-K), the tail without
dh (bcnf_grad_reduce) and dh alone (bcnf_stack_dh), HIP events around back-to-back launches.
Usage: python tools/tail_bench.py [--batch 4096] [--iters 50]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    from bench import FC_SMALL
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL).cuda()
    st = m.fused
    B = args.batch
    y = torch.randn(B, 19, device="cuda")
    h = torch.randn(B, 80, device="cuda")
    L = N.lib()
    stream = N.stream_handle(y.device)
    z, _, vals, (ws, pk) = st.launch_nll_forward(y, h, True, finalize=False)
    _, sb = st.workspace_bytes(B, True)
    slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device="cuda")
    N.check(L.bcnf_nll_backward(st._pdesc, N.ptr(pk), N.ptr(h), N.ptr(z), None, ctypes.c_int64(B), ctypes.c_int32(1),
                                N.ptr(ws), None, None, None, N.ptr(slab), None, None, None, stream), "bwd")
    dh = torch.empty_like(h)
    dp = torch.empty_like(st.flat)
    calls = {
        "tail": lambda: L.bcnf_backward_tail(st._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(h), N.ptr(ws), ctypes.c_int64(B),
                                             ctypes.c_int32(1), N.ptr(dh), N.ptr(dp), stream),
        "reduce+dw1h": lambda: L.bcnf_grad_reduce(st._pdesc, N.ptr(slab), N.ptr(h), N.ptr(ws), ctypes.c_int64(B),
                                                  ctypes.c_int32(1), N.ptr(dp), stream),
        "dh": lambda: L.bcnf_stack_dh(st._pdesc, N.ptr(pk), N.ptr(ws), ctypes.c_int64(B), ctypes.c_int32(1), N.ptr(dh),
                                      stream),
    }
    ref = None
    for name, fn in calls.items():
        N.check(fn(), name)
        torch.cuda.synchronize()
        if name == "tail":
            ref = (dp.clone(), dh.clone())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:12s} {e0.elapsed_time(e1) * 1e3 / args.iters:8.2f} us")
    print("slab bytes", sb, "equal after roles:", torch.equal(ref[0], dp), torch.equal(ref[1], dh))


if __name__ == "__main__":
    main()

"""Folded-feature-Linear launch timing (FC_small): pack vs pack+fold, the unfolded backward tail vs the folded one
(tail + Gx reduce + finish), HIP events around back-to-back launches on the launch stream.
Usage: python tools/fold_bench.py [--batch 4096] [--iters 50]"""
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
    lin = m.feature_network_stack.feature_networks[1].nn[0]
    wf, bf = lin.weight.detach(), lin.bias.detach()
    B = args.batch
    X = wf.shape[1]
    y = torch.randn(B, 19, device="cuda")
    x = torch.randn(B, X, device="cuda")
    xpad = torch.zeros(B, (X + 3) // 4 * 4, device="cuda")
    xpad[:, :X] = x
    xp = xpad[:, :X]                      # TrainStep's padded pool rows (float4 loads)
    h = torch.randn(B, wf.shape[0], device="cuda")
    L = N.lib()
    stream = N.stream_handle(y.device)
    _, _, _, (ws_h, pk_h) = st.launch_nll_forward(y, h, True, finalize=False)
    _, _, _, (ws, pk) = st.launch_fold_nll_forward(y, x, wf, bf, True, finalize=False)
    fold = torch.empty(N.query_i64(L.bcnf_fold_bytes, st._pdesc, ctypes.c_int32(X)) // 4, device="cuda")
    _, sb = st.workspace_bytes(B, True)
    slab_h = torch.empty(max(sb // 4, 1), device="cuda")
    fsb = N.query_i64(L.bcnf_fold_slab_bytes, st._pdesc, ctypes.c_int32(X), ctypes.c_int64(B))
    slab = torch.empty(max(fsb // 4, 1), device="cuda")
    z = torch.empty_like(y)
    for p, s, hh, w in ((pk_h, slab_h, h, ws_h), (pk, slab, x, ws)):
        N.check(L.bcnf_nll_backward(st._pdesc, N.ptr(p), N.ptr(hh), N.ptr(z), None, ctypes.c_int64(B),
                                    ctypes.c_int32(1), N.ptr(w), None, None, None, N.ptr(s), None, None, None, stream),
                "bwd")
    dh = torch.empty_like(h)
    dp = torch.empty_like(st.flat)
    dwf, dbf = torch.empty_like(wf), torch.empty_like(bf)
    calls = {
        "pack": lambda: L.bcnf_pack_params(st._pdesc, N.ptr(st.flat), N.ptr(st.qflat), N.ptr(pk_h), stream),
        "pack+fold": lambda: L.bcnf_pack_params_fold(st._pdesc, N.ptr(st.flat), N.ptr(st.qflat), N.ptr(wf), N.ptr(bf),
                                                     ctypes.c_int32(X), N.ptr(pk), N.ptr(fold), None, stream),
        "tail": lambda: L.bcnf_backward_tail(st._pdesc, N.ptr(pk_h), N.ptr(slab_h), N.ptr(h), N.ptr(ws_h),
                                             ctypes.c_int64(B), ctypes.c_int32(1), N.ptr(dh), N.ptr(dp), stream),
        "fold tail": lambda: L.bcnf_fold_backward_tail(st._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(x), ctypes.c_int32(X),
                                                       ctypes.c_int32(X),
                                                       N.ptr(wf), N.ptr(bf), N.ptr(ws), ctypes.c_int64(B),
                                                       ctypes.c_int32(1), N.ptr(dp), N.ptr(dwf), N.ptr(dbf), None, stream),
        "fold tail pad": lambda: L.bcnf_fold_backward_tail(st._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(xp),
                                                           ctypes.c_int32(xp.stride(0)), ctypes.c_int32(X), N.ptr(wf),
                                                           N.ptr(bf), N.ptr(ws), ctypes.c_int64(B), ctypes.c_int32(1),
                                                           N.ptr(dp), N.ptr(dwf), N.ptr(dbf), None, stream),
    }
    for name, fn in calls.items():
        N.check(fn(), name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:12s} {e0.elapsed_time(e1) * 1e3 / args.iters:8.2f} us", flush=True)


if __name__ == "__main__":
    main()

"""FusedAdam step and the clip after it, timed alone (HIP events) at FC_large's parameter shapes: the 48.86M-float
coupling flat buffer plus the feature MLP's 16 tensors. Usage: python tools/opt_bench.py [--iters 30]
(BCNF_AMD_LIB selects the library.)"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    from bcnf_amd.optim import FusedAdam
    sizes = [48_856_020 - 2_052_200] + [90 * 310, 310] + [310 * 310, 310] * 6 + [310 * 1360, 1360]
    g = torch.Generator(device="cuda").manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(n, device="cuda", generator=g) * 0.01) for n in sizes]
    for p in params:
        p.grad = torch.randn(p.shape, device="cuda", generator=g)
    opt = FusedAdam(params, lr=2e-4)
    nbytes_adam = sum(sizes) * 4 * 7          # g, p, m, v read; p, m, v written
    nbytes_clip = sum(sizes) * 4 * 2
    res = {"adam": [], "clip": []}
    for it in range(args.iters + 3):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        opt.step(defer_step_count=True)
        e[1].record()
        opt.clip_grad_norm_after_step(1.0)
        e[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            res["adam"].append(e[0].elapsed_time(e[1]) * 1e3)
            res["clip"].append(e[1].elapsed_time(e[2]) * 1e3)
    lib = os.environ.get("BCNF_AMD_LIB", "default")
    for k, v in res.items():
        v.sort()
        med = v[len(v) // 2]
        nb = nbytes_adam if k == "adam" else nbytes_clip
        print(f"{lib} {k}: median {med:.1f} us ({nb / med / 1e6:.2f} TB/s), min {v[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()

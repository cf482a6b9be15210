"""Wide-family weight pack (bcnf_wide_pack) timed alone at FC_large / LSTM_large shapes, beside a plain device copy of
the same byte count (the copy rate this box reaches). Usage: python tools/pack_bench.py [--iters 50]
(BCNF_AMD_LIB selects the library, as everywhere.)"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bench import FC_LARGE, LSTM_LARGE
    lib = os.environ.get("BCNF_AMD_LIB", "default")
    for name, cfg in (("fc_large", FC_LARGE), ("lstm_large", LSTM_LARGE)):
        torch.manual_seed(0)
        st = CondRealNVP_v2.from_config(cfg).cuda().fused
        out = torch.empty_like(st.packed())
        us = timed(lambda: st._pack_into(out), args.iters)
        ref = st.packed().clone()
        st._pack_into(out)
        same = bool(torch.equal(out, ref))
        # bytes the pack must move: every packed float written once, every source parameter read once
        nbytes = out.numel() * 4 + st.flat.numel() * 4
        src = torch.empty(nbytes // 8, dtype=torch.float32, device="cuda")
        dst = torch.empty_like(src)
        cu = timed(lambda: dst.copy_(src), args.iters)
        print(f"{name} {lib}: pack {us:.1f} us ({nbytes / us / 1e6:.2f} TB/s of packed-write + param-read bytes); "
              f"device copy of the same bytes {cu:.1f} us ({nbytes / cu / 1e6:.2f} TB/s); repack identical {same}",
              flush=True)


if __name__ == "__main__":
    main()

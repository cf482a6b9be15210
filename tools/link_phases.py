"""Phase timing of a forward link launch (workgroup 0, s_memtime stamps; bcnf_wide_debug_phases).
Usage (GPU box): python tools/link_phases.py [--batch 2048]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    from bench import FC_LARGE
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_LARGE).cuda().train()
    st = m.fused
    y = torch.randn(args.batch, 19, device="cuda")
    h = torch.randn(args.batch, 1360, device="cuda")
    dbg = torch.zeros(8, dtype=torch.int64, device="cuda")
    st.launch_nll_forward(y, h, True)
    torch.cuda.synchronize()
    N.lib().bcnf_wide_debug_phases(N.ptr(dbg))
    st.launch_nll_forward(y, h, True)      # the stamps of the last link launch of the pass remain
    torch.cuda.synchronize()
    N.lib().bcnf_wide_debug_phases(None)
    t = dbg.cpu().tolist()
    names = ["staged", "tail dots", "tail reduce", "coupling", "head vector", "head rows"]
    print("s_memtime deltas (shader clock cycles; last tail+head link launch of a training forward):")
    for i, n in enumerate(names):
        print(f"  {n:12s} {t[i + 1] - t[i]:8d}")
    print(f"  total        {t[6] - t[0]:8d}")


if __name__ == "__main__":
    main()

"""Wide-family micro-benchmark (FC_large shapes): a few forward (save) + backward passes of the coupling stack, for
rocprofv3 --pmc runs filtered to one kernel. Usage: python tools/kbench_wide.py [--batch 2048] [--iters 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    from bcnf_amd import CondRealNVP_v2
    from bench import FC_LARGE
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_LARGE).cuda().train()
    st = m.fused
    B = args.batch
    y = torch.randn(B, 19, device="cuda")
    h = torch.randn(B, 1360, device="cuda")
    for _ in range(args.iters):
        z, _, vals, saved = st.launch_nll_forward(y, h, True)
        st.launch_nll_backward(h, z, None, True, saved, want_dy=False, want_dh=True)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()

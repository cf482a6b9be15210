"""Per-launch device times of the NLL training pass (FusedStack.time_kernels) for the library named by
BCNF_AMD_LIB (A/B of experiment builds): python tools/abk.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bcnf_amd import CondRealNVP_v2
    from bench import FC_SMALL
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL).cuda().train()
    y = torch.randn(4096, 19, device="cuda")
    h = torch.randn(4096, 80, device="cuda")
    m.flat_parameters()
    t = m.fused.time_kernels(y, h, training=True, iters=50)
    print(os.environ.get("BCNF_AMD_LIB", "default"), {k: round(v, 2) for k, v in t.items()})


if __name__ == "__main__":
    main()

"""Device times of the folded training pass's launches (FusedStack.time_kernels with fold) for the library named by
BCNF_AMD_LIB, plus the forward's phase stamps when that build has them: python tools/raw_probe.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    from bench import FC_SMALL
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL).cuda().train()
    m.flat_parameters()
    B = 4096
    y = torch.randn(B, 19, device="cuda")
    x = torch.randn(B, 90, device="cuda")
    lin = m.feature_network_stack.feature_networks[1].nn[0]
    t = m.fused.time_kernels(y, None, training=True, iters=50, fold=(x, lin.weight.detach(), lin.bias.detach()))
    print(os.environ.get("BCNF_AMD_LIB", "default"), os.environ.get("BCNF_FOLD_RAW", "1"),
          {k: round(v, 2) for k, v in t.items()})
    L = N.lib()
    if hasattr(L, "bcnf_debug_phases"):
        buf = (ctypes.c_ulonglong * 32)()
        L.bcnf_debug_phases(buf)
        print("  fwd compute prologue/chain/wait", buf[8], buf[9], buf[10], " helper prologue/work/wait", buf[12],
              buf[13], buf[14])
        print("  prologue: compute at barrier0 / past it", buf[11] & 0xffffffff, buf[11] >> 32,
              " helper at barrier0 / barrier1", buf[15] & 0xffffffff, buf[15] >> 32)
        print("  compute: x/Wf landed", buf[16], " helper: table landed", buf[20], "gathers landed", buf[21],
              "records written", buf[22])
        print("  bwd compute prologue/chain/barrier-wait", buf[0], buf[1], buf[2],
              " helper barrier-wait/load-issue/grad-jobs/prep-store", buf[4], buf[5], buf[6], buf[7])
        if buf[25]:
            print(f"  compute wave: {buf[24]} cycles in {buf[25] * 10 / 1e3:.2f} us -> {buf[24] / buf[25] / 10:.3f} GHz;"
                  f" helper wave: {buf[26]} cycles in {buf[27] * 10 / 1e3:.2f} us")


if __name__ == "__main__":
    main()

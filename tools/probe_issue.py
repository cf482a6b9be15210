"""Driver of tools/probe_issue.hip: cycles per instruction (median over waves) for each instruction kind at one
and two waves per SIMD. Prints one line per (kind, layout)."""
import ctypes
import os

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "probe_issue.so"))
dev = torch.device("cuda")
inp = torch.rand(128, device=dev) * 0.01
cyc = torch.zeros(256 * 16, dtype=torch.int64, device=dev)
out = torch.zeros(256 * 512, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
names = ["fmac x4 indep", "fmac_dpp 2 acc", "fmac_dpp 4 acc", "fmac dependent", "v_exp indep", "v_pk_fma indep", "add_dpp 2 acc", "permlane16_swap", "combine chain"]
import sys
kinds = [int(k) for k in sys.argv[1:]] or list(range(len(names)))
for kind in kinds:
    name = names[kind]
    for threads, active in ((256, 4), (512, 4), (512, 8)):
        for _ in range(3):
            cyc.zero_()
            rc = lib.probe_run(kind, threads, active, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(cyc.data_ptr()),
                               ctypes.c_void_p(out.data_ptr()), st)
            torch.cuda.synchronize()
            assert rc == 0, rc
        c = cyc.view(256, 16)[:, :active].flatten().float()
        per = c.median().item() / (64 * 32)
        print(f"{name:16s} threads={threads} active_waves={active} ({active // 4} per SIMD): "
              f"{per:.2f} cycles/instr per wave", flush=True)

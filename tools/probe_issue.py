"""Driver of tools/probe_issue.hip: per instruction kind, at one and two waves per SIMD, the median over waves of
  * s_memtime ticks per instruction,
  * ns per instruction from s_memrealtime (a constant 100 MHz clock),
  * the implied shader clock d memtime / d realtime x 100 MHz (MI355X_MICROARCH.md note (6)),
after >= 2 s of back-to-back launches (the chip's clock settles under load). Prints one line per (kind, layout)."""
import ctypes
import os
import sys
import time

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "probe_issue.so"))
dev = torch.device("cuda")
inp = torch.rand(128, device=dev) * 0.01
cyc = torch.zeros(256 * 16 * 2, dtype=torch.int64, device=dev)
out = torch.zeros(256 * 512, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
# (name, instructions per body)
kinds_all = {0: ("fmac x4 indep", 32), 1: ("fmac_dpp 2 acc", 32), 2: ("fmac_dpp 4 acc", 32), 3: ("fmac dependent", 32),
             4: ("v_exp indep", 32), 5: ("v_pk_fma indep", 32), 6: ("add_dpp 2 acc", 32), 7: ("permlane16_swap", 32),
             8: ("combine chain", 32), 9: ("GELU dep chain", 34), 10: ("dense layer dpp", 38),
             11: ("dpp 2acc ror++", 32), 12: ("dpp rot16x2", 32), 13: ("dpp 1acc ror++", 32), 14: ("dpp 4acc ror++", 32),
             15: ("dpp 2acc ror1", 32), 16: ("fmac 2acc", 32),
             17: ("xdpp banks 23|1|0", 32), 18: ("xdpp acc=src bank", 32), 19: ("xdpp w=src bank", 32),
             20: ("xdpp acc0=w bank", 32), 21: ("xdpp all bank 2", 32), 22: ("xfmac all bank 2", 32),
             23: ("xfmac banks 23|1|0", 32)}
REP = 4096
kinds = [int(k) for k in sys.argv[1:]] or list(kinds_all)


def run(kind, threads, active):
    rc = lib.probe_run(kind, threads, active, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(cyc.data_ptr()),
                       ctypes.c_void_p(out.data_ptr()), st)
    assert rc == 0, rc


# warm the clock: >= 2 s of back-to-back launches
t0 = time.time()
while time.time() - t0 < 2.5:
    for _ in range(20):
        run(0, 512, 8)
    torch.cuda.synchronize()
for kind in kinds:
    name, n = kinds_all[kind]
    for threads, active in ((256, 4), (512, 4), (512, 8)):
        for _ in range(3):
            cyc.zero_()
            run(kind, threads, active)
            torch.cuda.synchronize()
        c = cyc.view(256, 16, 2)[:, :active].reshape(-1, 2).double()
        tick = c[:, 0].median().item() / (REP * n)
        ns = c[:, 1].median().item() * 10.0 / (REP * n)
        ghz = (c[:, 0] / c[:, 1].clamp(min=1)).median().item() * 0.1
        print(f"{name:16s} threads={threads} active_waves={active} ({active // 4} per SIMD): {tick:6.2f} memtime ticks, "
              f"{ns:6.3f} ns per instr per wave; memtime clock {ghz:5.3f} GHz -> {ns * ghz:5.2f} shader cycles",
              flush=True)

"""Folded vs unfolded wide NLL gradients (training / eval), per parameter: max|g|, max|diff|, run-to-run spread."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from conftest import load_golden  # noqa: E402
import test_gpu_configs as T  # noqa: E402

d = load_golden("g11_fc_large.npz")
m, sd = T._build(T.FC_LARGE_CFG, T.SEED + 15, T.SEED + 16)
m = m.to("cuda")
y = torch.from_numpy(d["y"]).cuda()
traj = torch.from_numpy(d["traj"]).cuda()
for mode in ("train", "eval"):
    getattr(m, mode)()
    st = m.fused.rng_state().clone()
    res = []
    for fold in (True, False, False):
        m.fused.rng_state().copy_(st)
        torch.manual_seed(11)
        res.append(T._nll_and_grads(m, y, traj, fold))
    (vf, gf), (vu, gu), (vu2, gu2) = res
    print(mode, "vals", vf.tolist(), vu.tolist(), vu2.tolist())
    for n in gf:
        print(f"{mode} {n:60s} max|g|={gu[n].abs().max():.3e} fold-unf={(gf[n]-gu[n]).abs().max():.3e} "
              f"unf-unf={(gu2[n]-gu[n]).abs().max():.3e}")

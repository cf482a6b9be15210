"""Diagnose the smoke's TrainStep step: loss of one eager fused step on a fresh / pre-used FC_small model."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bcnf_amd import CondRealNVP_v2, inn_nll_loss
from bcnf_amd.train import TrainStep

cfg = {"global": {"parameter_selection": [f"p{i}" for i in range(19)]},
       "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 7, "n_conditions": 80, "n_blocks": 32,
                            "dropout": 0.383, "act_norm": True}},
       "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                            {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
for pre in (False, True):
    for B in (64, 4096):
        torch.manual_seed(2024_03_25)
        model = CondRealNVP_v2.from_config(cfg).to("cuda:0")
        gen = torch.Generator().manual_seed(1)
        y = torch.randn(B, 19, generator=gen).cuda()
        traj = torch.randn(B, 30, 3, generator=gen).cuda()
        if pre:
            model.eval()
            z, h = model(y, traj, log_det_J=True, return_features=True)
            inn_nll_loss(z, model.log_det_J).backward()
            model.train()
            z2 = model(y, traj, log_det_J=True)
            inn_nll_loss(z2, model.log_det_J).backward()
        else:
            model.train()
        with torch.no_grad():
            z3 = model(y, traj, log_det_J=True)
            ref = inn_nll_loss(z3, model.log_det_J).item()
        vals = model.nll_loss(y, traj)
        print(f"pre={pre} B={B} unfused-train nll={ref:.5f} fused nll_loss={vals.tolist()}", flush=True)
        ts = TrainStep(model, lr=2e-4, capture=False)
        print("  TrainStep step:", ts.step(y, traj), flush=True)
        print("  TrainStep step 2:", ts.step(y, traj), flush=True)

"""Which config difference makes the pack-free forward's loss NaN (feature dropout kwarg / parameter names)."""
import copy, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bcnf_amd import CondRealNVP_v2

base = {"global": {"parameter_selection": [f"p{i}" for i in range(19)]},
        "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 7, "n_conditions": 80, "n_blocks": 32,
                             "dropout": 0.383, "act_norm": True}},
        "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                             {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
variants = {"smoke": base}
v = copy.deepcopy(base); v["feature_networks"][1]["kwargs"]["dropout"] = 0.244; variants["feat_dropout"] = v
for name, cfg in variants.items():
    for train in (False, True):
        torch.manual_seed(2024_03_25)
        m = CondRealNVP_v2.from_config(cfg).to("cuda:0").train(train)
        lin = m.feature_network_stack.feature_networks[1]
        gen = torch.Generator().manual_seed(1)
        y = torch.randn(64, 19, generator=gen).cuda()
        traj = torch.randn(64, 30, 3, generator=gen).cuda()
        for raw in (True, False):
            m.fused.use_raw_forward = raw
            print(name, "train" if train else "eval", "raw" if raw else "pack", m.nll_loss(y, traj).tolist(), flush=True)
    print(lin, flush=True)

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


# FC_small run config (configs/runs/old/trajectory_FC_small.yaml) as from_config sees it; identical to
# tests/golden/make_golden.py's FC_SMALL.
FC_SMALL_CFG = {
    "global": {"parameter_selection": ['x0_x', 'x0_y', 'x0_z', 'v0_x', 'v0_y', 'v0_z', 'g', 'w_x', 'w_y', 'w_z',
                                       'b', 'm', 'a_x', 'a_y', 'a_z', 'r', 'A', 'Cd', 'rho']},
    "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 7, "n_conditions": 80, "n_blocks": 32,
                         "dropout": 0.383, "act_norm": True}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
        {"type": "FullyConnected", "kwargs": {"sizes": [90, 80], "dropout": 0.244}},
    ],
}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name))


def golden_sd(d, prefix="sd/"):
    return {k[len(prefix):]: torch.from_numpy(np.ascontiguousarray(d[k])) for k in d.keys() if k.startswith(prefix)}


def close(a, b, rtol=1e-5, floor=1e-5):
    """The SURVEY §8d gate: |a-b| <= rtol*|b| + floor*max(1, max|b|)."""
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    scale = max(1.0, float(b.abs().max())) if b.numel() else 1.0
    err = (a - b).abs()
    ok = bool((err <= rtol * b.abs() + floor * scale).all())
    return ok, float(err.max()) if err.numel() else 0.0


@pytest.fixture(scope="session")
def g1():
    return load_golden("g1_fc_small.npz")

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


# configs/runs/old/trajectory_LSTM_large.yaml / trajectory_FC_large.yaml as from_config sees them (identical to
# tests/golden/make_golden.py's LSTM_LARGE / FC_LARGE)
LSTM_LARGE_CFG = {
    "global": FC_SMALL_CFG["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True, "layer": "Linear", "activation": "GELU",
                         "random_state": 2024_03_25}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 3}},
        {"type": "LSTM", "kwargs": {"input_size": 3, "hidden_size": 140, "output_size": 1360, "num_layers": 2,
                                    "dropout": 0.111, "bidirectional": True, "pooling": "mean"}},
    ],
}
FC_LARGE_CFG = {
    "global": FC_SMALL_CFG["global"],
    "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                         "dropout": 0.407, "act_norm": True}},
    "feature_networks": [
        {"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
        {"type": "FullyConnected", "kwargs": {"sizes": [90] + [310] * 7 + [1360], "dropout": 0.111}},
    ],
}


def large_proxy_sd(model, seed):
    """tests/golden/make_golden.py:large_proxy_state -- numpy PCG64 weights in state_dict order (the orthonormal
    matrices are kept), so full-depth fixtures need no 195 MB weight file."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for k, v in model.state_dict().items():
        if k.endswith("orthonormal_matrix"):
            sd[k] = v.detach().cpu().numpy()
            continue
        shape = tuple(v.shape)
        if k.endswith(".scale"):
            a = rng.uniform(0.7, 1.3, size=shape)
        elif len(shape) == 2:
            a = rng.uniform(-1.0, 1.0, size=shape) / np.sqrt(shape[1])
        else:
            a = rng.uniform(-0.05, 0.05, size=shape)
        sd[k] = a.astype(np.float32)
    return sd


@pytest.fixture(autouse=True)
def _lds_poison(request):
    """BCNF_LDS_POISON=1: every GPU test starts with every CU's LDS filled with NaN (bcnf_lds_fill), so a kernel that
    reads LDS it did not write shows up as a non-finite result instead of depending on what ran before."""
    import os
    if os.environ.get("BCNF_LDS_POISON") != "1" or request.node.get_closest_marker("gpu") is None:
        yield
        return
    import ctypes
    import torch
    from bcnf_amd import _native as N
    dev = torch.device("cuda", torch.cuda.current_device())
    N.check(N.lib().bcnf_lds_fill(ctypes.c_float(float("nan")), N.stream_handle(dev)), "bcnf_lds_fill")
    yield

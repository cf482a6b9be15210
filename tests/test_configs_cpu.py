"""Construction-level parity of the two wide BASELINE configs on CPU (no kernels run): trajectory_LSTM_large
(configs[3]) and trajectory_FC_large (configs[2]) build with the reference's state_dict layout, and
LSTM_large's `random_state` reseeds every orthonormal mix to the same Q, bit-identical to the reference's
(cnf.py:319-320, 410; fixture g10 made by running psaegert/bcnf, tests/golden/make_golden.py)."""
import copy

import numpy as np
import pytest
import torch

from conftest import FC_LARGE_CFG, LSTM_LARGE_CFG, large_proxy_sd, load_golden


@pytest.fixture(scope="module")
def lstm_model():
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(2024_03_25 + 12)
    return CondRealNVP_v2.from_config(LSTM_LARGE_CFG)


def test_lstm_large_identical_q_bit_exact(lstm_model):
    d = load_golden("g10_lstm_large.npz")
    qs = [v for k, v in lstm_model.state_dict().items() if k.endswith("orthonormal_matrix")]
    assert len(qs) == int(d["n_q"]) == 25 and bool(d["q_all_identical"])
    for q in qs:
        assert np.array_equal(q.numpy(), d["q"])            # every block: the reference's Q, byte for byte


def test_lstm_large_state_dict_layout(lstm_model):
    sd = lstm_model.state_dict()
    keys = [k for k in sd if k.startswith("feature_network_stack.")]
    assert keys[:2] == ["feature_network_stack.feature_networks.1.lstm.weight_ih_l0",
                        "feature_network_stack.feature_networks.1.lstm.weight_hh_l0"]
    assert tuple(sd["feature_network_stack.feature_networks.1.lstm.weight_ih_l1_reverse"].shape) == (560, 280)
    assert tuple(sd["feature_network_stack.feature_networks.1.linear.weight"].shape) == (1360, 280)
    assert sum(v.numel() for v in sd.values()) == 48_852_615           # SURVEY §8a-1 [measured]
    proxy = large_proxy_sd(lstm_model, 2024_03_25 + 13)
    assert proxy.keys() == sd.keys()


def test_lstm_pool_dim_option():
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(LSTM_LARGE_CFG)
    cfg["feature_networks"][1]["kwargs"]["pool_dim"] = 1
    cfg["model"]["kwargs"]["n_blocks"] = 2
    m = CondRealNVP_v2.from_config(cfg)
    fn = m.feature_network_stack.feature_networks[1]
    assert fn.pool_dim == 1
    with torch.no_grad():
        h = m.feature_network_stack(torch.randn(7, 30, 3))
    assert tuple(h.shape) == (7, 1360)                       # pooled over time: one row per sample


def test_fc_large_param_count():
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_LARGE_CFG)
    assert sum(v.numel() for v in m.state_dict().values()) == 48_865_045   # SURVEY §8a-1 [measured]

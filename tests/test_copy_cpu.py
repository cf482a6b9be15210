"""copy.deepcopy / pickle of a CondRealNVP_v2: the copy rebuilds its own fused stack over its
copied parameters (every coupling Parameter a view of the COPY's flat buffer), keeps the state_dict, the gradient
mode and the dropout seed, and its fused feature networks bind to the copy, not to the original."""
import copy
import io
import pickle

import torch

from conftest import FC_LARGE_CFG, FC_SMALL_CFG


def _views_of(model):
    flat = model.fused.flat
    lo, hi = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
    return all(lo <= p.data_ptr() < hi for p in model.fused.trainable)


def test_deepcopy_rebuilds_the_fused_stack():
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
    m.flat_parameters()
    m.fused.set_seed(77)
    c = copy.deepcopy(m)
    assert c.fused is not m.fused and c.fused.flat.data_ptr() != m.fused.flat.data_ptr()
    assert _views_of(c) and _views_of(m)
    assert c.fused.grad_mode == "flat" and c.fused.seed == 77
    for (k, a), (k2, b) in zip(m.state_dict().items(), c.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    with torch.no_grad():                       # the copy's parameters are its own
        c.layers[1].nn_a.nn[0].weight.add_(1.0)
    assert not torch.equal(c.layers[1].nn_a.nn[0].weight, m.layers[1].nn_a.nn[0].weight)


def test_deepcopy_binds_feature_rng_to_the_copy():
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.feature_network import _RNG_OWNERS
    cfg = copy.deepcopy(FC_LARGE_CFG)
    cfg["model"]["kwargs"]["n_blocks"] = 2
    torch.manual_seed(1)
    m = CondRealNVP_v2.from_config(cfg)
    c = copy.deepcopy(m)
    fm = m.feature_network_stack.feature_networks[1]
    fc = c.feature_network_stack.feature_networks[1]
    assert _RNG_OWNERS[fm]() is m and _RNG_OWNERS[fc]() is c
    pickle.loads(pickle.dumps(fc))              # no reference to a model inside the module's state


def test_torch_save_load_whole_model():
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(2)
    m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
    buf = io.BytesIO()
    torch.save(m, buf)
    buf.seek(0)
    d = torch.load(buf, weights_only=False)     # our own file, written just above
    assert _views_of(d) and torch.equal(d.fused.flat, m.fused.flat)

"""GPU tests of the fused feature-MLP layer (bcnf_linear_gelu_forward / _backward): FullyConnectedFeatureNetwork runs
each Linear -> GELU -> Dropout group of feature_network.py:128-134 as ONE launch, and its backward from the saved
derivative factors inside the dX / dW GEMMs.

Eval mode is checked against torch's own modules (fp32) and float64 gradients; training mode statistically (keep
rate, inverted-dropout scale, the saved factor equal to GELU' on kept units and 0 on dropped ones) and for
reproducibility from the same device Philox state (the owning model's coupling state)."""
import copy

import pytest
import torch
from torch import nn

from conftest import FC_LARGE_CFG, close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(sizes=(90, 310, 310, 1360), dropout=0.111, seed=3):
    from bcnf_amd.feature_network import FullyConnectedFeatureNetwork
    torch.manual_seed(seed)
    return FullyConnectedFeatureNetwork(list(sizes), dropout=dropout)


def _modules_forward(net, x):
    """The same network through torch's own modules (nn.Linear math, nn.GELU, nn.Dropout), no fusion."""
    for m in net.nn:
        x = nn.functional.linear(x, m.weight, m.bias) if isinstance(m, nn.Linear) else m(x)
    return x


@pytest.mark.parametrize("rows", [1, 37, 2048])
def test_fused_eval_matches_modules_and_fp64_gradients(rows):
    net = _net().to(DEV).eval()
    x = torch.randn(rows, 30, 3, generator=torch.Generator().manual_seed(rows)).to(DEV)
    with torch.no_grad():
        got = net(x)
        ref = _modules_forward(net, x.view(rows, -1))
    ok, err = close(got.cpu(), ref.cpu(), rtol=1e-5, floor=1e-5)
    assert ok, err
    # gradients of a scalar of the output vs float64 on the host
    w = torch.randn(rows, 1360, generator=torch.Generator().manual_seed(7))
    net.zero_grad(set_to_none=True)
    xg = x.clone().requires_grad_(True)
    (net(xg) * w.to(DEV)).sum().backward()
    n64 = copy.deepcopy(net).cpu().double()
    x64 = x.cpu().double().requires_grad_(True)
    (_modules_forward(n64, x64.view(rows, -1)) * w.double()).sum().backward()
    ok, err = close(xg.grad.cpu(), x64.grad, rtol=1e-4, floor=1e-4)
    assert ok, ("dx", err)
    for (name, p), (_, p64) in zip(net.named_parameters(), n64.named_parameters()):
        ok, err = close(p.grad.cpu(), p64.grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)


def test_fused_training_dropout_statistics_and_reproducibility():
    from bcnf_amd import _native as N
    net = _net(sizes=(64, 512, 8), dropout=0.25).to(DEV).train()
    lin = net.nn[0]
    x = torch.randn(4096, 64, device=DEV)
    rng = net.rng_state(x.device)
    st = rng.clone()
    a1 = net.run(x, upto=3)
    rng.copy_(st)
    a2 = net.run(x, upto=3)
    assert torch.equal(a1, a2)                                 # same device state -> same masks
    rng[1] += 1
    a3 = net.run(x, upto=3)
    assert not torch.equal(a1, a3)                             # the next offset draws fresh masks
    with torch.no_grad():
        pre = nn.functional.linear(x, lin.weight, lin.bias)
        ref = nn.functional.gelu(pre)
    kept = a1 != 0
    rate = kept.float().mean().item()
    assert abs(rate - 0.75) < 0.01, rate
    ok, err = close(a1[kept].cpu(), (ref[kept] / 0.75).cpu(), rtol=1e-5, floor=1e-5)
    assert ok, err
    # the saved factor: mask * GELU'(pre)
    rows, k, n = x.shape[0], 64, 512
    a = torch.empty(rows, n, device=DEV)
    g = torch.empty(rows, n, device=DEV)
    rng.copy_(st)
    N.check(N.lib().bcnf_linear_gelu_forward(N.ptr(x), N.ptr(lin.weight), N.ptr(lin.bias), rows, k, n, 0.25,
                                             N.ptr(rng), 0, N.ptr(a), N.ptr(g), N.stream_handle(x.device)), "fwd")
    assert torch.equal(a, a1)
    pre_d = pre.double()
    dgelu = 0.5 * (1 + torch.erf(pre_d / 2 ** 0.5)) + pre_d * torch.exp(-pre_d ** 2 / 2) / (2 * torch.pi) ** 0.5
    ok, err = close(g[kept].cpu(), (dgelu[kept] / 0.75).cpu(), rtol=1e-5, floor=1e-5)
    assert ok, err
    assert (g[~kept] == 0).all()


def test_model_feature_dropout_follows_coupling_state():
    """Inside CondRealNVP_v2 the feature dropout draws from the coupling's device Philox state: restoring
    model.fused.rng_state() replays the whole training step (feature and coupling masks) bit for bit."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(FC_LARGE_CFG)
    cfg["model"]["kwargs"]["n_blocks"] = 2
    torch.manual_seed(2)
    m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
    fn = m.feature_network_stack.feature_networks[1]
    y = torch.randn(300, 19, device=DEV)
    traj = torch.randn(300, 30, 3, device=DEV)
    assert fn.rng_state(y.device) is m.fused.rng_state()
    st = m.fused.rng_state().clone()
    v1 = m.nll_loss(y, traj).detach().clone()
    m.fused.rng_state().copy_(st)
    v2 = m.nll_loss(y, traj).detach().clone()
    assert torch.equal(v1, v2)
    v3 = m.nll_loss(y, traj).detach().clone()               # the finalize advanced the offset
    assert not torch.equal(v1, v3)


@pytest.mark.parametrize("owner", ["coupling_dropout_0", "standalone", "owner_eval"])
def test_feature_dropout_advances_without_coupling_dropout(owner):
    """with coupling dropout 0 (the coupling launches never bump the shared offset), a standalone
    feature network, or an owner not in training mode, the feature network advances the Philox offset itself after its
    last fused dropout layer, so consecutive training steps draw fresh feature masks."""
    from bcnf_amd import CondRealNVP_v2
    x = torch.randn(256, 30, 3, device=DEV)
    if owner == "standalone":
        fn = _net().to(DEV).train()
        run = lambda: fn(x)                                         # noqa: E731
    else:
        cfg = copy.deepcopy(FC_LARGE_CFG)
        cfg["model"]["kwargs"].update(n_blocks=2, dropout=0.0 if owner == "coupling_dropout_0" else 0.407)
        torch.manual_seed(4)
        m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
        fn = m.feature_network_stack.feature_networks[1]
        fn.train()
        if owner == "owner_eval":
            m.eval()
            fn.train()                                              # the feature dropout alone stays on
        y = torch.randn(256, 19, device=DEV)
        run = lambda: m.nll_loss(y, x) if owner == "coupling_dropout_0" else fn(x)   # noqa: E731
    # the feature activations of two consecutive steps
    acts = []
    for _ in range(2):
        off0 = int(fn.rng_state(x.device)[1].item())
        run()
        torch.cuda.synchronize()
        acts.append(fn.run(x.view(x.shape[0], -1), upto=3).detach().clone())
        # run() above advanced the offset too (one bump per run), so the step itself advanced it exactly once
        assert int(fn.rng_state(x.device)[1].item()) == off0 + 2
    assert not torch.equal(acts[0], acts[1])


def test_deepcopy_feature_dropout_follows_the_copy():
    """a deep-copied model's feature dropout draws from the COPY's coupling Philox state, so
    copy.fused.set_seed / a state restore on the copy cover its feature masks, and the original is untouched."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(FC_LARGE_CFG)
    cfg["model"]["kwargs"]["n_blocks"] = 2
    torch.manual_seed(5)
    m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
    c = copy.deepcopy(m)
    fm = m.feature_network_stack.feature_networks[1]
    fc = c.feature_network_stack.feature_networks[1]
    x = torch.randn(64, 90, device=DEV)
    assert fc.rng_state(x.device) is c.fused.rng_state()
    assert fm.rng_state(x.device) is m.fused.rng_state()
    assert fc.rng_state(x.device) is not fm.rng_state(x.device)
    c.fused.set_seed(1234)
    st = c.fused.rng_state().clone()
    a1 = fc.run(x, upto=3)
    m_state = m.fused.rng_state().clone()
    c.fused.rng_state().copy_(st)
    a2 = fc.run(x, upto=3)
    assert torch.equal(a1, a2)
    assert torch.equal(m.fused.rng_state(), m_state)              # the original's offset never moved
    import pickle
    pickle.loads(pickle.dumps(fc))                                  # no weakref inside the module's state


def test_standalone_feature_calls_of_a_training_owner_draw_fresh_masks():
    """with the owner training and coupling dropout on, the feature network leaves the offset
    advance to the coupling launch of the step. Called on its own twice (no coupling launch in between) it must still
    draw fresh masks, and a normal step (feature draw + coupling launch) still advances the offset exactly once."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(FC_LARGE_CFG)
    cfg["model"]["kwargs"]["n_blocks"] = 2
    torch.manual_seed(6)
    m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
    fn = m.feature_network_stack.feature_networks[1]
    x = torch.randn(256, 30, 3, device=DEV)
    y = torch.randn(256, 19, device=DEV)
    m.nll_loss(y, x)                                            # a step: feature draw, then the coupling's
    off0 = int(fn.rng_state(x.device)[1].item())
    a1 = fn(x).detach().clone()
    a2 = fn(x).detach().clone()                                 # no coupling launch since a1's draw
    assert not torch.equal(a1, a2)
    assert int(fn.rng_state(x.device)[1].item()) == off0 + 1    # advanced once, at a2's draw
    for _ in range(2):                                          # steps: exactly one advance each
        o = int(fn.rng_state(x.device)[1].item())
        m.nll_loss(y, x)
        torch.cuda.synchronize()
        assert int(fn.rng_state(x.device)[1].item()) == o + 1 + (1 if _ == 0 else 0)

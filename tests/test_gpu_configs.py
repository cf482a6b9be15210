"""GPU parity of the two wide BASELINE configs at FULL depth (26 blocks, 48.9M parameters) against the reference's
own outputs -- fixtures made by running psaegert/bcnf (tests/golden/make_golden.py, numpy-PCG64 weights loaded into
the reference's model, so no weight file is needed) -- and their gradients against the fp64 oracle.

* trajectory_LSTM_large (configs[3]): the reference pools its biLSTM+Linear output over the BATCH axis
  (feature_network.py:174), so it only runs at B = 30 (= the trajectory length); `pool_dim=0` reproduces that
  (g10: h, z, ldj, inverse). The documented fix `pool_dim=1` pools over time; g10's h1 / z1 / ldj1 are the
  reference's own LSTM and Linear modules pooled that way at B = 48 -- config-4 parity at the h boundary.
* trajectory_FC_large (configs[2]): g11 (FC[90, 310 x 7, 1360] feature net, B = 48).

Gates: values |got - ref| <= 1e-5 |ref| + 1e-5 max(1, max|ref|) (north star); gradients 1e-4 vs fp64.
"""
import copy
import math

import numpy as np
import pytest
import torch

from conftest import FC_LARGE_CFG, LSTM_LARGE_CFG, close, large_proxy_sd, load_golden
from oracle import cnf_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 2024_03_25


def _build(cfg, init_seed, weight_seed, pool_dim=None):
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(cfg)
    if pool_dim is not None:
        cfg["feature_networks"][1]["kwargs"]["pool_dim"] = pool_dim
    torch.manual_seed(init_seed)
    m = CondRealNVP_v2.from_config(cfg)
    sd = large_proxy_sd(m, weight_seed)
    if "random_state" in cfg["model"]["kwargs"]:
        # every block's Q is the reference's one reseeded Q (g10); pin it to the reference's bytes rather than this
        # host's LAPACK rounding of the same QR
        q = load_golden("g10_lstm_large.npz")["q"]
        for k in sd:
            if k.endswith("orthonormal_matrix"):
                ok, err = close(sd[k], q, rtol=0.0, floor=1e-6)
                assert ok, (k, err)
                sd[k] = np.ascontiguousarray(q)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    assert type(m.fused).__name__ == "WideStack"
    return m, sd


def _check_values(m, y, cond, d, keys=("h", "z", "ldj"), inv_key="inv"):
    with torch.no_grad():
        z, h = m.forward(y, cond, log_det_J=True, return_features=True)
        ldj = m.log_det_J.clone()
        lp = m.log_prob(y, cond)
    for name, got in zip(keys, (h, z, ldj)):
        ok, err = close(got.cpu(), d[name])
        assert ok, (name, err)
    zr = d[keys[1]].astype(np.float64)
    ref_lp = -(0.5 * (zr ** 2).sum(1) - d[keys[2]]) - 0.5 * 19 * math.log(2 * math.pi)
    ok, err = close(lp.cpu(), ref_lp)
    assert ok, ("log_prob", err)
    if inv_key:
        with torch.no_grad():
            inv = m.inverse(torch.from_numpy(d[keys[1]]).to(DEV), cond)
        ok, err = close(inv.cpu(), d[inv_key])
        assert ok, ("inverse", err)


@pytest.fixture(scope="module")
def lstm_pool_batch():
    m, _ = _build(LSTM_LARGE_CFG, SEED + 12, SEED + 13)
    return m.to(DEV).eval()


def test_lstm_large_pool_over_batch_matches_reference(lstm_pool_batch):
    """configs[3] as the reference runs it (B = 30, h pooled over the batch axis): h, z, ldj, log_prob, inverse."""
    d = load_golden("g10_lstm_large.npz")
    y, traj = torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["traj"]).to(DEV)
    _check_values(lstm_pool_batch, y, traj, d)


def test_lstm_large_pool_dim1_matches_reference_modules():
    """The pool_dim=1 fix at B = 48: h (the h boundary), z, ldj, log_prob vs the reference's own modules."""
    d = load_golden("g10_lstm_large.npz")
    m, _ = _build(LSTM_LARGE_CFG, SEED + 12, SEED + 13, pool_dim=1)
    m.to(DEV).eval()
    y, traj = torch.from_numpy(d["y1"]).to(DEV), torch.from_numpy(d["traj1"]).to(DEV)
    _check_values(m, y, traj, d, keys=("h1", "z1", "ldj1"), inv_key=None)


def test_lstm_large_pool_dim1_gradients_vs_fp64():
    """pool_dim=1, eval, full depth: dL/dh at the h boundary (the HIP backward's output into the LSTM), every
    coupling gradient and every LSTM / Linear gradient vs the same step in fp64 (oracle flow + torch LSTM)."""
    from bcnf_amd import inn_nll_loss
    d = load_golden("g10_lstm_large.npz")
    m, sd = _build(LSTM_LARGE_CFG, SEED + 12, SEED + 13, pool_dim=1)
    y0, t0 = torch.from_numpy(d["y1"][:24]), torch.from_numpy(d["traj1"][:24])
    # fp64 reference: the feature module in double on CPU (a copy), the flow through the oracle
    fref = copy.deepcopy(m.feature_network_stack).double().eval()
    h64 = fref(t0.double())
    h64.retain_grad()
    spec = O.StackSpec(size=19, nested_sizes=[526] * 5, n_blocks=26, n_conditions=1360, dropout=0.407,
                       act_norm=True)
    sdg = {k: torch.from_numpy(np.ascontiguousarray(v)).double().requires_grad_(not k.endswith("orthonormal_matrix"))
           for k, v in sd.items() if k.startswith("layers.")}
    zo, lo = O.model_forward(sdg, spec, y0.double(), h64)
    O.inn_nll_loss(zo, lo).backward()
    m.to(DEV).eval()
    m.zero_grad(set_to_none=True)
    # MIOpen's RNN backward refuses eval mode; torch's own LSTM kernels (same math) take it
    with torch.backends.cudnn.flags(enabled=False):
        z, h = m.forward(y0.to(DEV), t0.to(DEV), log_det_J=True, return_features=True)
        h.retain_grad()
        inn_nll_loss(z, m.log_det_J).backward()
    ok, err = close(h.grad.cpu(), h64.grad, rtol=1e-4, floor=1e-4)
    assert ok, ("dL/dh", err)
    named_ref = dict(fref.named_parameters())
    n = 0
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ref = sdg[name].grad if name.startswith("layers.") else named_ref[name[len("feature_network_stack."):]].grad
        ok, err = close(p.grad.cpu(), ref, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    assert n == sum(1 for k in sd if not k.endswith("orthonormal_matrix"))


@pytest.fixture(scope="module")
def fc_large():
    d = load_golden("g11_fc_large.npz")
    m, sd = _build(FC_LARGE_CFG, SEED + 15, SEED + 16)
    # The seeded construction reproduces every Q up to the host LAPACK's QR rounding (bit-exact on the host that
    # generated g11; a few ulps on other CPUs), so the flow runs on the reference's own Q matrices.
    for k in sd:
        if k.endswith("orthonormal_matrix"):
            ok, err = close(sd[k], d["q/" + k], rtol=0.0, floor=1e-6)
            assert ok, (k, err)
            sd[k] = np.ascontiguousarray(d["q/" + k])
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    return m.to(DEV).eval(), sd, d


def test_fc_large_full_depth_matches_reference(fc_large):
    """configs[2] at full depth (26 blocks, FC[90, 310 x 7, 1360]): h, z, ldj, log_prob, inverse."""
    m, _, d = fc_large
    _check_values(m, torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["traj"]).to(DEV), d)


def test_fc_large_full_depth_gradients_vs_fp64(fc_large):
    """Every parameter gradient (flow and the 8-layer feature MLP) and dL/dy vs the fp64 oracle, eval mode."""
    from bcnf_amd import inn_nll_loss
    m, sd, d = fc_large
    spec = O.StackSpec(size=19, nested_sizes=[526] * 5, n_blocks=26, n_conditions=1360, dropout=0.407,
                       act_norm=True, feature_sizes=[90] + [310] * 7 + [1360], feature_dropout=0.111)
    sdg = {k: torch.from_numpy(np.ascontiguousarray(v)).double().requires_grad_(not k.endswith("orthonormal_matrix"))
           for k, v in sd.items()}
    y = torch.from_numpy(d["y"][:24]).double().requires_grad_(True)
    traj = torch.from_numpy(d["traj"][:24])
    zo, lo = O.model_forward(sdg, spec, y, O.feature_forward(sdg, spec, traj.double()))
    O.inn_nll_loss(zo, lo).backward()
    m.zero_grad(set_to_none=True)
    yd = y.detach().float().to(DEV).requires_grad_(True)
    z = m.forward(yd, traj.to(DEV), log_det_J=True)
    inn_nll_loss(z, m.log_det_J).backward()
    ok, err = close(yd.grad.cpu(), y.grad, rtol=1e-4, floor=1e-4)
    assert ok, ("dL/dy", err)
    n = 0
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ok, err = close(p.grad.cpu(), sdg[name].grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    assert n == sum(1 for k in sd if not k.endswith("orthonormal_matrix"))


def _nll_and_grads(m, y, cond, fold):
    m.fold_features = fold
    try:
        m.zero_grad(set_to_none=True)
        with torch.backends.cudnn.flags(enabled=False):
            vals = m.nll_loss(y, cond)
            vals[0].backward()
        with torch.no_grad():      # after the step: the probe runs the feature layers (and their dropout RNG)
            assert (m._wide_fold(y, (cond,)) is not None) == fold
    finally:
        del m.fold_features
    return vals.detach().cpu(), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()
                                 if p.grad is not None}


def test_fc_large_folded_nll_gradients_vs_fp64(fc_large):
    """The training path (nll_loss) with the feature MLP's last Linear (310 -> 1360) folded into the condition
    projection (bcnf_wide_fold_*): loss and every gradient vs the fp64 oracle, and vs the unfolded launch."""
    m, sd, d = fc_large
    spec = O.StackSpec(size=19, nested_sizes=[526] * 5, n_blocks=26, n_conditions=1360, dropout=0.407,
                       act_norm=True, feature_sizes=[90] + [310] * 7 + [1360], feature_dropout=0.111)
    sdg = {k: torch.from_numpy(np.ascontiguousarray(v)).double().requires_grad_(not k.endswith("orthonormal_matrix"))
           for k, v in sd.items()}
    y = torch.from_numpy(d["y"][:24])
    traj = torch.from_numpy(d["traj"][:24])
    zo, lo = O.model_forward(sdg, spec, y.double(), O.feature_forward(sdg, spec, traj.double()))
    loss64 = O.inn_nll_loss(zo, lo)
    loss64.backward()
    vf, gf = _nll_and_grads(m, y.to(DEV), traj.to(DEV), True)
    vu, gu = _nll_and_grads(m, y.to(DEV), traj.to(DEV), False)
    ok, err = close(vf[:1], loss64.detach().reshape(1))
    assert ok, ("loss", err)
    assert set(gf) == set(gu) and len(gf) == sum(1 for k in sd if not k.endswith("orthonormal_matrix"))
    for name in gf:
        ok, err = close(gf[name], sdg[name].grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, "vs fp64", err)
        ok, err = close(gf[name], gu[name], rtol=1e-4, floor=1e-4)
        assert ok, (name, "vs unfolded", err)


def test_fc_large_folded_training_mode_equals_unfolded(fc_large):
    """Training mode (feature dropout 0.111, coupling dropout 0.407): the folded and unfolded launches draw the same
    masks from the same torch / Philox states and agree on the loss and every gradient."""
    m, _, d = fc_large
    y = torch.from_numpy(d["y"]).to(DEV)
    traj = torch.from_numpy(d["traj"]).to(DEV)
    m.train()
    try:
        st = m.fused.rng_state().clone()
        torch.manual_seed(11)
        vf, gf = _nll_and_grads(m, y, traj, True)
        m.fused.rng_state().copy_(st)
        torch.manual_seed(11)
        vu, gu = _nll_and_grads(m, y, traj, False)
    finally:
        m.eval()
    ok, err = close(vf, vu, rtol=1e-5, floor=1e-5)
    assert ok, ("vals", err)
    for name in gf:
        ok, err = close(gf[name], gu[name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)


def test_lstm_large_pool_dim1_folded_nll_equals_unfolded():
    """pool_dim=1 LSTM_large: mean over time commutes with the last Linear (280 -> 1360), which folds into the
    projection; loss and every gradient (LSTM included) agree with the unfolded launch."""
    d = load_golden("g10_lstm_large.npz")
    m, _ = _build(LSTM_LARGE_CFG, SEED + 12, SEED + 13, pool_dim=1)
    m.to(DEV).eval()
    y, traj = torch.from_numpy(d["y1"]).to(DEV), torch.from_numpy(d["traj1"]).to(DEV)
    vf, gf = _nll_and_grads(m, y, traj, True)
    vu, gu = _nll_and_grads(m, y, traj, False)
    ok, err = close(vf, vu, rtol=1e-5, floor=1e-5)
    assert ok, ("vals", err)
    assert set(gf) == set(gu)
    for name in gf:
        ok, err = close(gf[name], gu[name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)


# ---------------------------------------------------------------------------------------------------------------------
# The wide training step at the BENCH batch sizes (FC_large B = 2048 per GPU, LSTM_large B = 1024), so the GEMM cost
# model's large-M tilings (tiling W on 96 x 48 / 48 x 48, K slices, XCD-contiguous grids; engaged only at M >= 1024)
# run through the fused ACT / GRAD / LINGRAD epilogues and the fold's condition GEMMs, not only the plain-store hook.
# nb = 2 blocks keep the fp64 oracle at a few seconds of host time; every per-block kernel is the full-width one.
def _bench_shape(cfg, pool_dim=None, n_blocks=2):
    cfg = copy.deepcopy(cfg)
    cfg["model"]["kwargs"]["n_blocks"] = n_blocks
    cfg["model"]["kwargs"].pop("random_state", None)
    if pool_dim is not None:
        cfg["feature_networks"][1]["kwargs"]["pool_dim"] = pool_dim
    return cfg


def _bench_inputs(B, lstm, seed=31):
    g = torch.Generator().manual_seed(seed)
    y = torch.randn(B, 19, generator=g)
    traj = torch.randn(B, 30, 3, generator=g)
    return y, traj


def _fp64_step(m, sd, cfg, y, traj, lstm):
    """Loss, z, ldj and every gradient of the eval NLL step in float64 on the host: the oracle's flow, the oracle's
    FC feature MLP (FC_large) or torch's own LSTM + Linear in double (LSTM_large, pool over time)."""
    kw = cfg["model"]["kwargs"]
    sdg = {k: torch.from_numpy(np.ascontiguousarray(v)).double().requires_grad_(not k.endswith("orthonormal_matrix"))
           for k, v in sd.items()}
    if lstm:
        spec = O.StackSpec(size=19, nested_sizes=kw["nested_sizes"], n_blocks=kw["n_blocks"],
                           n_conditions=kw["n_conditions"], dropout=kw["dropout"], act_norm=True)
        fref = copy.deepcopy(m.feature_network_stack).double().eval()
        h64 = fref(traj.double())
        named = {"feature_network_stack." + n: p for n, p in fref.named_parameters()}
    else:
        fk = cfg["feature_networks"][1]["kwargs"]
        spec = O.StackSpec(size=19, nested_sizes=kw["nested_sizes"], n_blocks=kw["n_blocks"],
                           n_conditions=kw["n_conditions"], dropout=kw["dropout"], act_norm=True,
                           feature_sizes=fk["sizes"], feature_dropout=fk["dropout"])
        h64 = O.feature_forward(sdg, spec, traj.double())
        named = {}
    zo, lo = O.model_forward({k: v for k, v in sdg.items() if k.startswith("layers.")} if lstm else sdg, spec,
                             y.double(), h64)
    loss = O.inn_nll_loss(zo, lo)
    loss.backward()
    grads = {k: v.grad for k, v in sdg.items() if v.grad is not None}
    grads.update({k: p.grad for k, p in named.items() if p.grad is not None})
    return loss.detach(), zo.detach(), lo.detach(), grads


@pytest.mark.parametrize("which,B", [("fc_large", 2048), ("lstm_large", 1024)])
def test_wide_bench_batch_step_vs_fp64(which, B):
    """configs[2] / [3] shapes at the bench's per-GPU batch: z, ldj (1e-5 gate), the folded NLL loss and every
    gradient -- coupling, fold, feature MLP / LSTM -- against float64 (1e-4), on the cost model's own tilings."""
    lstm = which == "lstm_large"
    cfg = _bench_shape(LSTM_LARGE_CFG if lstm else FC_LARGE_CFG, pool_dim=1 if lstm else None)
    m, sd = _build(cfg, SEED + 41, SEED + 42)
    y, traj = _bench_inputs(B, lstm)
    loss64, z64, l64, g64 = _fp64_step(m, sd, cfg, y, traj, lstm)
    m.to(DEV).eval()
    yd, td = y.to(DEV), traj.to(DEV)
    with torch.no_grad():
        z = m.forward(yd, td, log_det_J=True)
        ldj = m.log_det_J.clone()
    for name, got, ref in (("z", z, z64), ("ldj", ldj, l64)):
        ok, err = close(got.cpu(), ref)
        assert ok, (name, err)
    m.zero_grad(set_to_none=True)
    with torch.backends.cudnn.flags(enabled=False):      # MIOpen's RNN backward refuses eval mode
        vals = m.nll_loss(yd, td)
        vals[0].backward()
        with torch.no_grad():
            assert m._wide_fold(yd, (td,)) is not None   # the folded training path ran
    ok, err = close(vals[:1].detach().cpu(), loss64.reshape(1))
    assert ok, ("loss", err)
    n = 0
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ok, err = close(p.grad.cpu(), g64[name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    assert n == len(g64) == sum(1 for k in sd if not k.endswith("orthonormal_matrix"))


@pytest.mark.parametrize("which,B", [("fc_large", 2048), ("lstm_large", 1024)])
def test_wide_bench_batch_training_fused_equals_unfolded(which, B):
    """Training mode at the bench batch (feature dropout, coupling dropout 0.407): the fused (folded) step and the
    unfolded launches draw the same masks from the same torch / Philox states and agree on the loss and every
    gradient."""
    lstm = which == "lstm_large"
    cfg = _bench_shape(LSTM_LARGE_CFG if lstm else FC_LARGE_CFG, pool_dim=1 if lstm else None)
    m, _ = _build(cfg, SEED + 43, SEED + 44)
    y, traj = _bench_inputs(B, lstm, seed=37)
    m.to(DEV).train()
    yd, td = y.to(DEV), traj.to(DEV)
    st = m.fused.rng_state().clone()
    torch.manual_seed(5)
    vf, gf = _nll_and_grads(m, yd, td, True)
    m.fused.rng_state().copy_(st)
    torch.manual_seed(5)
    vu, gu = _nll_and_grads(m, yd, td, False)
    ok, err = close(vf, vu, rtol=1e-5, floor=1e-5)
    assert ok, ("vals", err)
    assert set(gf) == set(gu)
    for name in gf:
        ok, err = close(gf[name], gu[name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)

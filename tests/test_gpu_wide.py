"""GPU parity of the wide-MLP coupling family (trajectory_FC_large / trajectory_LSTM_large class, bcnf_wide.hip)
against the reference's own outputs (fixture g7: FC_large-shaped proxy, C = 1360, nested_sizes = [526] * 5, made by
running psaegert/bcnf, tests/golden/make_golden.py) and against the CPU oracle (oracle/cnf_oracle.py).

Tolerances as tests/test_gpu_parity.py: values |got - ref| <= 1e-5 |ref| + 1e-5 max(1, max|ref|); gradients
1e-4 (fp64 oracle as the reference there, since fp32 rounding of a 1,370-term sum is itself ~1e-6 relative).
"""
import math

import numpy as np
import pytest
import torch

from conftest import close, load_golden
from oracle import cnf_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
SEED = 2024_03_25


def _lib():
    from bcnf_amd import _native as N
    return N


# ------------------------------------------------------------------------------------------ GEMM tiles
@pytest.mark.parametrize("tiling", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
@pytest.mark.parametrize("layout", [0, 1, 2, 3])
@pytest.mark.parametrize("mnk", [(64, 64, 32), (100, 70, 36), (2048, 528, 528), (18, 527, 300), (1030, 1360, 64),
                                 (3, 5, 4), (300, 200, 2052),
                                 # 176 x 176 with unpredicated staging loads (whole K tiles, grid inside the padded rows):
                                 # an exact 2 x 2 grid, and the hidden-Linear gradient's own shape (M = H, N = H + 1, K = B)
                                 (352, 352, 64), (526, 527, 2048)])
def test_wide_gemm_layouts_vs_fp64(layout, mnk, tiling):
    """C = A B through the MFMA tile machinery (tiling 0 = the dispatcher's choice, 1 = 128x128 32x32-MFMA,
    2 = 64x64, 3 = 128x48 16x16-MFMA, 4 = the same on 8 waves, 5 = 96x48 on 6 waves, 6 = LDS-DMA tiling C,
    7 = tiling C large tiles, 8 = tiling C 48 x 48, 9 = 176 x 176 on 11 waves (strided x strided only; layout 2 at the
    last two shapes takes its unpredicated-load instance), 10 / 11 =
    tiling W 96 x 48 / 48 x 48 (LDS-resident B band, K-contiguous x K-contiguous with K <= 768 only); every operand
    layout; ragged M / N / K tails) vs fp64."""
    import ctypes
    N = _lib()
    M, Nn, K = mnk
    g = torch.Generator().manual_seed(M * 7 + Nn + K + layout)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    B = torch.randn(K, Nn, generator=g, dtype=torch.float64)
    ref = A @ B
    pad = lambda n: (n + 3) // 4 * 4  # noqa: E731
    if layout in (0, 1):  # A[m][k]
        Ad = torch.zeros(M, pad(K), dtype=torch.float32)
        Ad[:, :K] = A.float()
    else:                 # A[k][m]
        Ad = torch.zeros(pad(K), pad(M), dtype=torch.float32)
        Ad[:K, :M] = A.t().float()
    if layout in (0, 3):  # B[n][k]
        Bd = torch.zeros(Nn, pad(K), dtype=torch.float32)
        Bd[:, :K] = B.t().float()
    else:                 # B[k][n]
        Bd = torch.zeros(pad(K), pad(Nn), dtype=torch.float32)
        Bd[:K, :Nn] = B.float()
    Ad, Bd = Ad.to(DEV), Bd.to(DEV)
    C = torch.full((M, pad(Nn)), float("nan"), device=DEV)
    Kp = pad(K) if layout != 2 else K
    rc = N.lib().bcnf_wide_gemm_test(layout | (tiling << 4), M, Nn, Kp, N.ptr(Ad), Ad.shape[1], N.ptr(Bd), Bd.shape[1], N.ptr(C),
                                     C.shape[1], N.stream_handle(C.device))
    N.check(rc, "bcnf_wide_gemm_test")
    torch.cuda.synchronize()
    got = C[:, :Nn].double().cpu()
    tol = 2e-6 * (A.abs() @ B.abs()) + 1e-6
    assert bool(((got - ref).abs() <= tol).all()), float((got - ref).abs().max())
    assert torch.isnan(C[:, Nn:]).all() or Nn == C.shape[1]      # nothing written past N


# ------------------------------------------------------------------------------------------ model builders
def _model(shape, seed=7, fsizes=None):
    from bcnf_amd import CondRealNVP_v2
    C = shape["n_conditions"]
    torch.manual_seed(seed)
    if fsizes is None:
        fnets = [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": C}}]
    else:
        fnets = [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": fsizes[0]}},
                 {"type": "FullyConnected", "kwargs": {"sizes": fsizes, "dropout": 0.0}}]
    cfg = {"global": {"parameter_selection": [f"p{i}" for i in range(shape["size"])]},
           "model": {"kwargs": shape}, "feature_networks": fnets}
    m = CondRealNVP_v2.from_config(cfg)
    assert type(m.fused).__name__ == "WideStack"
    return m


def _perturb(m):
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("scale"):
                p.copy_(0.5 + torch.rand_like(p))
            elif n.endswith("bias") and n.count(".") == 2:
                p.copy_(0.1 * torch.randn_like(p))


def _spec(shape, fsizes=()):
    return O.StackSpec(size=shape["size"], nested_sizes=shape["nested_sizes"], n_blocks=shape["n_blocks"],
                       n_conditions=shape["n_conditions"], dropout=shape["dropout"], act_norm=shape["act_norm"],
                       two_way=shape.get("two_way", False), feature_sizes=list(fsizes))


WIDE_SHAPES = [
    dict(size=19, nested_sizes=[40] * 3, n_blocks=3, n_conditions=24, dropout=0.2, act_norm=True),
    dict(size=7, nested_sizes=[33] * 2, n_blocks=2, n_conditions=8, dropout=0.0, act_norm=False),
    dict(size=19, nested_sizes=[20], n_blocks=3, n_conditions=4, dropout=0.1, act_norm=True),      # one hidden layer
    dict(size=32, nested_sizes=[64] * 4, n_blocks=2, n_conditions=300, dropout=0.0, act_norm=True),
    dict(size=19, nested_sizes=[526] * 5, n_blocks=2, n_conditions=1360, dropout=0.407, act_norm=True),  # FC_large
    # two_way couplings (nn_a then nn_b per block, cnf.py:176-186; the reference's non-inverse inverse, :198-213)
    dict(size=19, nested_sizes=[40] * 2, n_blocks=3, n_conditions=24, dropout=0.2, act_norm=True, two_way=True),
    dict(size=7, nested_sizes=[33] * 3, n_blocks=2, n_conditions=6, dropout=0.0, act_norm=False, two_way=True),
    # n_conditions not a multiple of 4 (rows re-laid to 4-float multiples inside the library)
    dict(size=19, nested_sizes=[24] * 2, n_blocks=2, n_conditions=13, dropout=0.0, act_norm=True),
]


@pytest.fixture(params=[-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10],
                ids=["auto", "t128x128", "t64x64", "t128x48", "t128x48w8", "t96x48w6", "glds96x48", "glds_large",
                     "glds48x48", "t176x176w11", "wband96x48", "wband48x48"])
def tiling(request):
    """A forced GEMM tiling travels in the model's descriptor (BcnfStackDesc.gemm_tiling = t + 1): per call, no
    library-global setting."""
    return request.param


@pytest.mark.parametrize("shape", WIDE_SHAPES)
@pytest.mark.parametrize("B", [1, 37, 300])
def test_wide_shapes_vs_oracle(shape, B, tiling):
    """Forward / log-det / inverse / eval gradients of the wide family vs the oracle (fp64 for gradients), with every
    GEMM tiling (all epilogues: activation, gradient, Linear-gradient, row-mapped, plain)."""
    if tiling >= 0 and B == 1:
        pytest.skip("B = 1 covered by the auto tiling")
    _check_vs_oracle(shape, B, tiling)


@pytest.mark.parametrize("shape", [WIDE_SHAPES[0], WIDE_SHAPES[4]], ids=["wide40", "fc_large"])
def test_wide_link_grids_past_256_workgroups(shape):
    """B = 4100 rows: every link launch (forward, inverse, backward) has 513 workgroups, past the 256 at which the
    per-workgroup rotation of the links' weight staging (stage4x2) once stepped beyond the staged regions;
    the rotation only reorders the copy, so the results must match the oracle as at small B."""
    _check_vs_oracle(shape, 4100, -1)


def _check_vs_oracle(shape, B, tiling):
    from bcnf_amd import inn_nll_loss
    m = _model(shape)
    m.fused.desc.gemm_tiling = tiling + 1
    _perturb(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    spec = _spec(shape)
    m.to(DEV).eval()
    C = shape["n_conditions"]
    gen = torch.Generator().manual_seed(B)
    y = torch.randn(B, shape["size"], generator=gen)
    c = torch.randn(B, C, generator=gen)
    zr, lr = O.model_forward(sd, spec, y, c)
    z = m.forward(y.to(DEV), c.to(DEV), log_det_J=True)
    ok, err = close(z.detach().cpu(), zr)
    assert ok, ("z", err)
    ok, err = close(m.log_det_J.detach().cpu(), lr)
    assert ok, ("ldj", err)
    with torch.no_grad():
        lp = m.log_prob(y.to(DEV), c.to(DEV))
    assert close(lp.cpu(), O.log_prob(zr, lr))[0]
    zl = torch.randn(B, shape["size"], generator=gen)
    inv_r = O.model_inverse(sd, spec, zl, c)
    with torch.no_grad():
        inv = m.inverse(zl.to(DEV), c.to(DEV))
    ok, err = close(inv.cpu(), inv_r)
    assert ok, ("inverse", err)
    # eval-mode gradients (parameters, dL/dh, dL/dy) vs fp64 oracle autograd
    sdg = {k: v.double().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in sd.items()}
    cg = c.double().clone().requires_grad_(True)
    yg = y.double().clone().requires_grad_(True)
    zo, lo = O.model_forward(sdg, spec, yg, cg)
    O.inn_nll_loss(zo, lo).backward()
    m.zero_grad(set_to_none=True)
    cd = c.to(DEV).requires_grad_(True)
    yd = y.to(DEV).requires_grad_(True)
    zg = m.forward(yd, cd, log_det_J=True)
    inn_nll_loss(zg, m.log_det_J).backward()
    assert close(cd.grad.cpu(), cg.grad, rtol=1e-4, floor=1e-4)[0]
    assert close(yd.grad.cpu(), yg.grad, rtol=1e-4, floor=1e-4)[0]
    n = 0
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ok, err = close(p.grad.cpu(), sdg[name].grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    assert n == len([k for k in sd if not k.endswith("orthonormal_matrix")])


def _large_proxy_sd(model, seed=SEED):
    """tests/golden/make_golden.py:large_proxy_state (numpy PCG64 weights in state_dict order)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for k, v in model.state_dict().items():
        if k.endswith("orthonormal_matrix"):
            sd[k] = v.numpy()
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


@pytest.fixture(scope="module")
def g7_model():
    d = load_golden("g7_large_proxy.npz")
    shape = dict(size=19, nested_sizes=[526] * 5, n_blocks=2, n_conditions=1360, dropout=0.407, act_norm=True)
    m = _model(shape, fsizes=[90, 1360])
    sd = _large_proxy_sd(m)
    sd["layers.2.orthonormal_matrix"] = d["q/layers.2.orthonormal_matrix"]
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    m.to(DEV).eval()
    return m, d, {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}


def test_wide_g7_matches_reference(g7_model):
    """FC_large-shaped proxy (C = 1360, [526] * 5): z, log|det J|, log_prob and inverse vs the reference's outputs."""
    m, d, _ = g7_model
    y, traj = torch.from_numpy(d["y"]).to(DEV), torch.from_numpy(d["traj"]).to(DEV)
    with torch.no_grad():
        z = m.forward(y, traj, log_det_J=True)
        ldj = m.log_det_J.clone()
        lp = m.log_prob(y, traj)
        inv = m.inverse(torch.from_numpy(d["z"]).to(DEV), traj)
    ok, err = close(z.cpu(), d["z"])
    assert ok, ("z", err)
    ok, err = close(ldj.cpu(), d["ldj"])
    assert ok, ("ldj", err)
    ref_lp = -(0.5 * (d["z"].astype(np.float64) ** 2).sum(1) - d["ldj"]) - 0.5 * 19 * math.log(2 * math.pi)
    ok, err = close(lp.cpu(), ref_lp)
    assert ok, ("log_prob", err)
    ok, err = close(inv.cpu(), d["inv"])
    assert ok, ("inverse", err)


def test_wide_g7_grads_vs_oracle(g7_model):
    """FC_large-shaped proxy: every parameter gradient and dL/dy against the fp64 oracle."""
    from bcnf_amd import inn_nll_loss
    m, d, sd = g7_model
    spec = _spec(dict(size=19, nested_sizes=[526] * 5, n_blocks=2, n_conditions=1360, dropout=0.407,
                      act_norm=True), fsizes=[90, 1360])
    sdg = {k: v.double().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in sd.items()}
    y = torch.from_numpy(d["y"]).double().requires_grad_(True)
    h = O.feature_forward(sdg, spec, torch.from_numpy(d["traj"]).double())
    zo, lo = O.model_forward(sdg, spec, y, h)
    O.inn_nll_loss(zo, lo).backward()
    m.zero_grad(set_to_none=True)
    yd = torch.from_numpy(d["y"]).to(DEV).requires_grad_(True)
    z = m.forward(yd, torch.from_numpy(d["traj"]).to(DEV), log_det_J=True)
    inn_nll_loss(z, m.log_det_J).backward()
    assert close(yd.grad.cpu(), y.grad, rtol=1e-4, floor=1e-4)[0]
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ok, err = close(p.grad.cpu(), sdg[name].grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)


def _train_model(shape=None):
    shape = shape or dict(size=19, nested_sizes=[96] * 3, n_blocks=3, n_conditions=80, dropout=0.3, act_norm=True)
    m = _model(shape, fsizes=[90, 80])
    _perturb(m)
    return m.to(DEV).train()


def test_wide_nll_fused_equals_unfused_with_dropout():
    """Training mode: nll_loss (forward + per-sample NLL + finalize; backward through the NLL) == forward +
    inn_nll_loss + autograd on the same dropout stream; the finalize advances the RNG offset once."""
    from bcnf_amd import inn_nll_loss
    m = _train_model()
    m.flat_parameters()
    gen = torch.Generator().manual_seed(3)
    y = torch.randn(257, 19, generator=gen).to(DEV)
    traj = torch.randn(257, 30, 3, generator=gen).to(DEV)
    m.fused.set_seed(99)
    vals = m.nll_loss(y, traj)
    torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    g_fused = m.fused.flat_param.grad.clone()
    assert int(m.fused.rng_state()[1].item()) == 1
    m.zero_grad(set_to_none=True)
    m.fused.flat_param.grad = None
    m.fused.set_seed(99)
    z = m(y, traj, log_det_J=True)
    loss = inn_nll_loss(z, m.log_det_J)
    loss.backward()
    assert abs(loss.item() - vals[0].item()) <= 1e-6 * abs(loss.item())
    assert torch.allclose(m.fused.flat_param.grad, g_fused, rtol=1e-5, atol=1e-6)


def test_wide_dropout_statistics_and_fd_consistency():
    """Philox dropout keeps ~(1 - p) of the hidden units (from the saved derivative factors), fresh masks per
    call, and the backward is the exact gradient of the forward that drew them (central differences at a fixed
    RNG offset)."""
    from bcnf_amd import inn_nll_loss
    m = _train_model()
    st = m.fused
    st.set_seed(1234)
    gen = torch.Generator().manual_seed(5)
    y = torch.randn(512, 19, generator=gen).to(DEV)
    traj = torch.randn(512, 30, 3, generator=gen).to(DEV)
    with torch.no_grad():
        z1 = m(y, traj)
        z2 = m(y, traj)
        assert not torch.allclose(z1, z2)
        h = m.feature_network_stack(traj)
        _, _, _, (ws, _) = st.launch_forward(y, h, True, save=True)
    # G factors: region after P (B x nb x HP) and nllp (B) and A (nb x NH x B x HP); see carve() in bcnf_wide.hip
    B, nb, NH, H, HP = 512, 3, 3, 96, 100
    off = (B * nb * HP + 3) // 4 * 4 + 64
    off += (B + 3) // 4 * 4 + 64
    off += (nb * NH * B * HP + 3) // 4 * 4 + 64
    G = ws[off: off + nb * NH * B * HP].view(nb, NH, B, HP)[..., :H]
    keep = (G != 0).double().mean().item()
    assert abs(keep - 0.7) < 0.01, keep

    def loss_at(offset):
        st.rng_state()[1] = offset
        zz = m(y, traj, log_det_J=True)
        return inn_nll_loss(zz, m.log_det_J)

    m.zero_grad(set_to_none=True)
    L0 = loss_at(77)
    L0.backward()
    g = torch.cat([p.grad.reshape(-1) for p in st.trainable])
    gn = g.norm().item()
    v = g / gn
    eps = 1e-3 / max(1.0, gn / 100.0)
    with torch.no_grad():
        st.flat.add_(eps * v)
        Lp = loss_at(77).double().item()
        st.flat.add_(-2 * eps * v)
        Lm = loss_at(77).double().item()
        st.flat.add_(eps * v)
    fd = (Lp - Lm) / (2 * eps)
    assert abs(fd - gn) <= 2e-2 * gn, (fd, gn)
    with torch.no_grad():
        assert loss_at(78).item() != loss_at(77).item()


def test_wide_trainstep_graph_replay_equals_eager():
    """HIP-graph TrainStep on the wide family == eager TrainStep over 3 dropout steps, bit for bit, and the loss
    goes down over a few steps."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(11)
    pool_y = torch.randn(1024, 19, generator=gen).to(DEV)
    pool_t = torch.randn(1024, 30, 3, generator=gen).to(DEV)
    idxs = [torch.randperm(1024, generator=gen)[:256].to(DEV) for _ in range(3)]
    res = []
    for capture in (False, True):
        torch.manual_seed(0)
        m = _train_model()
        m.fused.set_seed(77)
        st = TrainStep(m, lr=2e-4, capture=capture)
        st.set_pool(pool_y, pool_t)
        losses = [st.step_indexed(i) for i in idxs]
        res.append((losses, [p.detach().clone() for p in m.parameters()], int(m.fused.rng_state()[1].item())))
    (l0, p0, r0), (l1, p1, r1) = res
    assert l0 == l1 and r0 == r1 == 3
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    torch.manual_seed(0)
    m = _train_model()
    st = TrainStep(m, lr=1e-3, capture=True)
    y, t = pool_y[:256], pool_t[:256]
    first = st.step(y, t)[0]
    for _ in range(20):
        last = st.step(y, t)[0]
    assert last < first, (first, last)


def test_wide_sample_matches_oracle():
    """sample(outer=True): the reference's CPU z stream and chunking, features once per condition (cond_index)."""
    shape = dict(size=19, nested_sizes=[48] * 2, n_blocks=3, n_conditions=80, dropout=0.2, act_norm=True)
    m = _model(shape, fsizes=[90, 80])
    _perturb(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m.to(DEV).eval()
    traj = torch.randn(7, 30, 3, generator=torch.Generator().manual_seed(2))
    torch.manual_seed(123)
    got = m.sample(50, traj, outer=True, batch_size=3, sample_batch_size=16)
    torch.manual_seed(123)
    ref = O.sample(sd, _spec(shape, fsizes=[90, 80]), 50, traj, outer=True, batch_size=3, sample_batch_size=16)
    assert got.shape == ref.shape == (50, 7, 19)
    ok, err = close(got, ref)
    assert ok, err


# ------------------------------------------------------------------------------------------ two_way vs the reference
def test_wide_two_way_coupling_layer_matches_reference():
    """Standalone two_way coupling (D = 7, nested [19] * 5, C = 5: fixture g6 from the reference) and the one-way
    layer at the reference test's shapes (tests/test_cnf.py:18-32): z, log|det J|, and the reference's inverse."""
    from bcnf_amd import ConditionalAffineCouplingLayer
    d = load_golden("g6_two_way.npz")
    x, c = torch.from_numpy(d["x"]).to(DEV), torch.from_numpy(d["c"]).to(DEV)
    for prefix, two_way, zk, lk, ik in (("layer_sd/", True, "z", "ldj", "inv"), ("l1_sd/", False, "z1", "ldj1", "inv1")):
        layer = ConditionalAffineCouplingLayer(input_size=7, nested_sizes=[19] * 5, n_conditions=5, two_way=two_way)
        layer.load_state_dict({k[len(prefix):]: torch.from_numpy(d[k]) for k in d.keys() if k.startswith(prefix)})
        layer.to(DEV).eval()
        with torch.no_grad():
            z = layer(x, c, log_det_J=True)
            inv = layer.inverse(z, c)
        for got, key in ((z, zk), (layer.log_det_J, lk), (inv, ik)):
            ok, err = close(got.cpu(), d[key])
            assert ok, (prefix, key, err)


def test_wide_two_way_model_matches_reference():
    """two_way CondRealNVP_v2 (D = 19, [16] * 3, C = 80, 4 blocks, ActNorm; fixture g6 from the reference): z, ldj,
    inverse; and every gradient vs the fp64 oracle."""
    from bcnf_amd import CondRealNVP_v2, inn_nll_loss
    from conftest import FC_SMALL_CFG
    d = load_golden("g6_two_way.npz")
    cfg = {"global": FC_SMALL_CFG["global"], "feature_networks": FC_SMALL_CFG["feature_networks"],
           "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 3, "n_conditions": 80, "n_blocks": 4,
                                "dropout": 0.0, "act_norm": True, "two_way": True}}}
    m = CondRealNVP_v2.from_config(cfg)
    assert type(m.fused).__name__ == "WideStack"
    sd = {k[len("m_sd/"):]: torch.from_numpy(d[k]) for k in d.keys() if k.startswith("m_sd/")}
    m.load_state_dict(sd)
    m.to(DEV).eval()
    y, traj = torch.from_numpy(d["m_y"]).to(DEV), torch.from_numpy(d["m_traj"]).to(DEV)
    with torch.no_grad():
        z = m(y, traj, log_det_J=True)
        ldj = m.log_det_J.clone()
        inv = m.inverse(z, traj)
    for got, key in ((z, "m_z"), (ldj, "m_ldj"), (inv, "m_inv")):
        ok, err = close(got.cpu(), d[key])
        assert ok, (key, err)
    spec = O.StackSpec(size=19, nested_sizes=[16] * 3, n_blocks=4, n_conditions=80, act_norm=True, two_way=True,
                       feature_sizes=[90, 80], feature_dropout=0.244)
    sdg = {k: v.double().clone().requires_grad_(not k.endswith("orthonormal_matrix")) for k, v in sd.items()}
    h = O.feature_forward(sdg, spec, torch.from_numpy(d["m_traj"]).double())
    zo, lo = O.model_forward(sdg, spec, torch.from_numpy(d["m_y"]).double(), h)
    O.inn_nll_loss(zo, lo).backward()
    m.zero_grad(set_to_none=True)
    zg = m(y, traj, log_det_J=True)
    inn_nll_loss(zg, m.log_det_J).backward()
    n = 0
    for name, p in m.named_parameters():
        if p.grad is None:
            continue
        ok, err = close(p.grad.cpu(), sdg[name].grad, rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    assert n == len([k for k in sd if not k.endswith("orthonormal_matrix")])


@pytest.mark.parametrize("two_way", [False, True], ids=["one_way", "two_way"])
def test_weight_pack_layout_is_the_parameter_relayout(two_way):
    """k_wpack_all (bcnf_wide_pack, one launch): every packed region equals the re-layout of the model's own
    parameters -- W0's condition columns as W0h rows, each hidden W row-major AND transposed, W0's y columns
    transposed, the last Linear, Q, the Linear-1 biases (bit-exact copies, zero padding) and the ActNorm log-det
    constants (within 1e-6). Two-way blocks are two virtual blocks (nn_a, then nn_b). Layout: WideLayout in
    bcnf_wide.hip."""
    from bcnf_amd import CondRealNVP_v2
    H, C, nb, NH, D = 40, 12, 3, 3, 19
    cfg = {"global": {"parameter_selection": [f"p{i}" for i in range(D)]},
           "model": {"kwargs": {"size": D, "nested_sizes": [H] * NH, "n_conditions": C, "n_blocks": nb,
                                "dropout": 0.0, "act_norm": True, "two_way": two_way}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": C}}]}
    torch.manual_seed(3)
    m = CondRealNVP_v2.from_config(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("scale"):
                p.copy_(0.5 + torch.rand_like(p))
    m.to(DEV)
    pk = m.fused.packed().cpu()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    Da, Db = (D + 1) // 2, D // 2
    S = 2 if two_way else 1
    nin, nout = [Da, Db], [Db, Da]
    r4 = lambda n: (n + 3) // 4 * 4  # noqa: E731
    HP, Cp, nv, WY, WL = r4(H + 1), r4(C), nb * S, Da, 2 * (Da if two_way else Db)
    o_w0h = 0
    o_hid = o_w0h + r4(nv * HP * Cp)
    o_hidT = o_hid + r4(nv * (NH - 1) * HP * HP)
    o_w0y = o_hidT + r4(nv * (NH - 1) * HP * HP)
    o_wl = o_w0y + r4(nv * WY * HP)
    o_q = o_wl + r4(nv * WL * HP)
    o_ldc = o_q + r4((nb - 1) * D * D)
    o_b0 = o_ldc + r4(nb)
    assert pk.numel() == o_b0 + nv * HP
    coup = [i for i in range(3 * nb) if any(k.startswith(f"layers.{i}.nn_a.") for k in sd)]
    an = [i for i in range(3 * nb) if f"layers.{i}.scale" in sd]
    qs = [i for i in range(3 * nb) if f"layers.{i}.orthonormal_matrix" in sd]
    assert len(coup) == nb and len(an) == nb - 1 and len(qs) == nb - 1
    for v in range(nv):
        li, side = coup[v // S], v % S
        pre = f"layers.{li}.nn_{'ab'[side]}.nn."
        wk = sorted((k for k in sd if k.startswith(pre) and k.endswith(".weight")), key=lambda k: int(k.split(".")[-2]))
        assert len(wk) == NH + 1
        W = [sd[k] for k in wk]
        b0 = sd[wk[0][:-len("weight")] + "bias"]
        ni, no = nin[side], nout[side]
        want = torch.zeros(HP, Cp)
        want[:H, :C] = W[0][:, ni:]
        assert torch.equal(pk[o_w0h + v * HP * Cp: o_w0h + (v + 1) * HP * Cp].view(HP, Cp), want), ("w0h", v)
        for l in range(1, NH):
            base = (v * (NH - 1) + l - 1) * HP * HP
            want = torch.zeros(HP, HP)
            want[:H, :H] = W[l]
            assert torch.equal(pk[o_hid + base: o_hid + base + HP * HP].view(HP, HP), want), ("hid", v, l)
            assert torch.equal(pk[o_hidT + base: o_hidT + base + HP * HP].view(HP, HP), want.t()), ("hidT", v, l)
        want = torch.zeros(WY, HP)
        want[:ni, :H] = W[0][:, :ni].t()
        assert torch.equal(pk[o_w0y + v * WY * HP: o_w0y + (v + 1) * WY * HP].view(WY, HP), want), ("w0y", v)
        want = torch.zeros(WL, HP)
        want[:2 * no, :H] = W[NH]
        assert torch.equal(pk[o_wl + v * WL * HP: o_wl + (v + 1) * WL * HP].view(WL, HP), want), ("wl", v)
        want = torch.zeros(HP)
        want[:H] = b0
        assert torch.equal(pk[o_b0 + v * HP: o_b0 + (v + 1) * HP], want), ("b0", v)
    for k, li in enumerate(qs):
        assert torch.equal(pk[o_q + k * D * D: o_q + (k + 1) * D * D].view(D, D), sd[f"layers.{li}.orthonormal_matrix"])
    for k in range(nb):
        want = float(torch.log(sd[f"layers.{an[k]}.scale"].abs()).sum()) if k < nb - 1 else 0.0
        assert abs(float(pk[o_ldc + k]) - want) <= 1e-6 * max(1.0, abs(want)), ("ldc", k)

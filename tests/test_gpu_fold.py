"""GPU tests of the folded linear feature network (bcnf_fold_train_forward, or bcnf_pack_params_fold +
bcnf_fold_nll_forward where its table does not apply, then bcnf_fold_backward_tail): model.nll_loss folds a single-Linear feature stack (trajectory_FC_small) into the
condition projection. Oracle: the same model with the fold switched off (fold_features = False: feature
Linear GEMM -> h -> projection -> dL/dh -> feature dW), itself pinned to the reference's golden fixture in
test_gpu_train.py. The fold computes the same sums reassociated, so the gate is fp32 rounding: loss within
2e-6 relative, gradients within rtol 1e-4 / atol 1e-5 of the unfolded path (their own tolerance vs the fp64
oracle is 1e-4 as well)."""
import copy
import ctypes
import math

import numpy as np
import pytest
import torch

from conftest import FC_SMALL_CFG, close, golden_sd

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(cfg, sd=None, train=False, seed=0):
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(seed)
    m = CondRealNVP_v2.from_config(cfg)
    if sd is not None:
        m.load_state_dict(sd)
    m.to(DEV)
    m.train(train)
    m.flat_parameters()
    return m


def _grads(m, y, traj, fold, seed):
    m.fold_features = fold
    m.zero_grad(set_to_none=True)
    m.fused.flat_param.grad = None
    m.fused.set_seed(seed)
    vals = m.nll_loss(y, traj)
    torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    lin = m.feature_network_stack.feature_networks[1].nn[0]
    return (vals.detach().clone(), m.fused.flat_param.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone(),
            int(m.fused.rng_state()[1].item()))


def _cfg(in_shape, C, nb=32):
    cfg = copy.deepcopy(FC_SMALL_CFG)
    cfg["model"]["kwargs"]["n_conditions"] = C
    cfg["model"]["kwargs"]["n_blocks"] = nb
    X = int(np.prod(in_shape))
    cfg["feature_networks"][0]["kwargs"]["output_size"] = X
    cfg["feature_networks"][1]["kwargs"]["sizes"] = [X, C]
    return cfg


def test_fold_is_taken_for_fc_small(g1):
    m = _model(FC_SMALL_CFG, golden_sd(g1))
    y = torch.randn(8, 19, device=DEV)
    traj = torch.randn(8, 30, 3, device=DEV)
    assert m._foldable_linear(y, (traj,)) is not None
    m.fold_features = False
    assert m._foldable_linear(y, (traj,)) is None


@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("B", [1, 37, 300, 4096])
def test_fold_equals_unfolded(g1, B, train):
    gen = torch.Generator().manual_seed(B)
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn(B, 30, 3, generator=gen).to(DEV)
    m = _model(FC_SMALL_CFG, golden_sd(g1), train=train)
    v1, g1_, w1, b1, r1 = _grads(m, y, traj, True, 1234)
    v0, g0, w0, b0, r0 = _grads(m, y, traj, False, 1234)
    assert r1 == r0 == (1 if train else 0)                 # same dropout stream, advanced once
    assert abs(v1[0].item() - v0[0].item()) <= 2e-6 * abs(v0[0].item()) + 1e-6
    assert v1[0].item() == v1[1].item() and v1[2].item() == 0.0
    for a, b, what in ((g1_, g0, "stack"), (w1, w0, "feature W"), (b1, b0, "feature b")):
        ok, err = close(a.cpu(), b.cpu(), rtol=1e-4, floor=1e-5)
        assert ok, (what, err)


def test_fold_matches_reference_golden(g1):
    """The folded pass against the reference's own loss and gradients (the g1 fixture)."""
    m = _model(FC_SMALL_CFG, golden_sd(g1))
    y = torch.from_numpy(np.ascontiguousarray(g1["y"])).to(DEV)
    traj = torch.from_numpy(np.ascontiguousarray(g1["traj"])).to(DEV)
    vals, g, gw, gb, _ = _grads(m, y, traj, True, 1)
    loss = float(g1["loss"])
    assert abs(vals[0].item() - loss) <= 2e-6 * abs(loss) + 1e-5
    named = dict(m.named_parameters())
    fp = m.fused
    g = g.cpu()
    for (off, k), p in zip(fp._offsets, fp.trainable):
        name = [kk for kk, vv in named.items() if vv is p][0]
        ok, err = close(g[off:off + k].view(p.shape), g1["grad/" + name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
    pre = "feature_network_stack.feature_networks.1.nn.0."
    for name, got in ((pre + "weight", gw), (pre + "bias", gb)):
        ok, err = close(got.cpu(), g1["grad/" + name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)


@pytest.mark.parametrize("in_shape,C,nb", [((20, 4), 80, 5), ((7, 3), 13, 3), ((79, 3), 96, 4)])
def test_fold_other_shapes(in_shape, C, nb):
    """X % 4 == 0 (vector loads), odd X / C, and X = 237 (Xp = 240, the largest split-K staging that fits LDS)."""
    cfg = _cfg(in_shape, C, nb)
    m = _model(cfg, train=True, seed=3)
    gen = torch.Generator().manual_seed(7)
    B = 333
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn((B,) + tuple(in_shape), generator=gen).to(DEV)
    assert m._foldable_linear(y, (traj,)) is not None
    v1, g1_, w1, b1, _ = _grads(m, y, traj, True, 99)
    v0, g0, w0, b0, _ = _grads(m, y, traj, False, 99)
    assert abs(v1[0].item() - v0[0].item()) <= 2e-6 * abs(v0[0].item()) + 1e-6
    for a, b, what in ((g1_, g0, "stack"), (w1, w0, "feature W"), (b1, b0, "feature b")):
        ok, err = close(a.cpu(), b.cpu(), rtol=1e-4, floor=1e-5)
        assert ok, (what, err)


def test_fold_trainstep_graph_equals_unfolded_eager(g1):
    """HIP-graph TrainStep on the folded path stays within rounding of the unfolded eager step."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(5)
    pool_y = torch.randn(512, 19, generator=gen).to(DEV)
    pool_t = torch.randn(512, 30, 3, generator=gen).to(DEV)
    idx = torch.randperm(512, generator=gen)[:256].to(DEV)
    out = []
    for fold, capture in ((False, False), (True, True)):
        m = _model(FC_SMALL_CFG, golden_sd(g1), train=True)
        m.fold_features = fold
        m.fused.set_seed(21)
        st = TrainStep(m, lr=2e-4, capture=capture)
        st.set_pool(pool_y, pool_t)
        losses = [st.step_indexed(idx) for _ in range(2)]
        out.append((losses, [p.detach().clone() for p in m.parameters()]))
    (l0, p0), (l1, p1) = out
    for a, b in zip(l0, l1):
        assert abs(a[0] - b[0]) <= 2e-6 * abs(b[0]) + 1e-6
    # Adam normalises each update to ~lr * sign(g): where |g| is near eps, fp32-rounding-level gradient
    # differences move a parameter by up to lr per step; everywhere else the replicas agree to 1e-6
    diff = torch.cat([(a - b).abs().reshape(-1) for a, b in zip(p0, p1)])
    assert diff.max().item() <= 2 * 2e-4 + 1e-6
    assert (diff > 1e-6).float().mean().item() < 1e-3


@pytest.mark.parametrize("train", [False, True])
def test_fold_padded_rows_equal_contiguous(g1, train):
    """x rows ldx = 92 floats apart (TrainStep's padded pool; float4 loads) give bit-identical results to contiguous
    rows, whatever the padding holds (NaN here: the columns beyond X are discarded by select)."""
    B = 333
    gen = torch.Generator().manual_seed(11)
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn(B, 30, 3, generator=gen).to(DEV)
    pad = torch.full((B, 92), float("nan"), device=DEV)
    pad[:, :90] = traj.reshape(B, 90)
    traj_p = pad[:, :90].view(B, 30, 3)
    assert traj_p.stride() == (92, 3, 1)
    m = _model(FC_SMALL_CFG, golden_sd(g1), train=train)
    assert m._foldable_linear(y, (traj_p,))[0].stride(0) == 92
    a = _grads(m, y, traj, True, 5)
    b = _grads(m, y, traj_p, True, 5)
    for u, v in zip(a[:4], b[:4]):
        assert torch.equal(u, v)


def test_trainstep_pads_fold_pool(g1):
    from bcnf_amd.train import TrainStep
    m = _model(FC_SMALL_CFG, golden_sd(g1), train=True)
    st = TrainStep(m, lr=2e-4, capture=False)
    gen = torch.Generator().manual_seed(2)
    st.set_pool(torch.randn(64, 19, generator=gen).to(DEV), torch.randn(64, 30, 3, generator=gen).to(DEV))
    assert st._pool[1].shape == (64, 92) and st._cond_shape == ((30, 3), 90)
    assert torch.count_nonzero(st._pool[1][:, 90:]) == 0
    m.fold_features = False
    st2 = TrainStep(m, lr=2e-4, capture=False)
    st2.set_pool(torch.randn(64, 19).to(DEV), torch.randn(64, 30, 3).to(DEV))
    assert st2._cond_shape is None and st2._pool[1].shape == (64, 30, 3)


@pytest.mark.parametrize("raw", [False, True])
@pytest.mark.parametrize("epoch", [False, True])
def test_gather_inside_pack_launch_is_exact(g1, epoch, raw):
    """The captured step's batch gather run inside the first launch (BcnfGather2: the pack launch, or the pack-free
    forward, which reads the pool rows itself and writes the gathered rows for the backward) == the separate
    gather launch: logged values, parameters and gradients bit for bit (index buffer and epoch-cursor forms)."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(31)
    py = torch.randn(600, 19, generator=gen).to(DEV)
    pt = torch.randn(600, 30, 3, generator=gen).to(DEV)
    order = torch.randperm(600, generator=gen)[:3 * 200].to(DEV)
    out = []
    for fuse in (False, True):
        m = _model(FC_SMALL_CFG, golden_sd(g1), train=True)
        m.fused.set_seed(3)
        m.fused.use_raw_forward = raw
        st = TrainStep(m, lr=2e-4)
        st.fuse_gather = fuse
        st.epoch_unroll = 2
        st.set_pool(py, pt)
        if epoch:
            st.set_epoch(order, 200)
            vals = st.run_epoch()
        else:
            vals = [st.step_indexed(order[i * 200:(i + 1) * 200]) for i in range(3)]
        out.append((vals, [p.detach().clone() for p in st.params], [p.grad.clone() for p in st.params]))
    (v0, p0, g0), (v1, p1, g1_) = out
    assert v0 == v1
    for a, b in zip(p0 + g0, p1 + g1_):
        assert torch.equal(a, b)


@pytest.mark.parametrize("train", [False, True])
def test_fold_without_feature_bias(g1, train):
    """A feature Linear without bias (bf = NULL through the fold kernels) == the unfolded path."""
    gen = torch.Generator().manual_seed(17)
    B = 257
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn(B, 30, 3, generator=gen).to(DEV)
    m = _model(FC_SMALL_CFG, golden_sd(g1), train=train)
    m.feature_network_stack.feature_networks[1].nn[0].bias = None
    out = []
    for fold in (True, False):
        m.fold_features = fold
        m.zero_grad(set_to_none=True)
        m.fused.flat_param.grad = None
        m.fused.set_seed(8)
        vals = m.nll_loss(y, traj)
        torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
        lin = m.feature_network_stack.feature_networks[1].nn[0]
        out.append((vals.detach().clone(), m.fused.flat_param.grad.clone(), lin.weight.grad.clone()))
    (v1, g1_, w1), (v0, g0, w0) = out
    assert abs(v1[0].item() - v0[0].item()) <= 2e-6 * abs(v0[0].item()) + 1e-6
    for a, b, what in ((g1_, g0, "stack"), (w1, w0, "feature W")):
        ok, err = close(a.cpu(), b.cpu(), rtol=1e-4, floor=1e-5)
        assert ok, (what, err)


def test_raw_forward_is_taken_for_fc_small(g1):
    m = _model(FC_SMALL_CFG, golden_sd(g1))
    assert m.fused.raw_table(90) is not None
    assert m.fused.raw_table(200) is None                   # X > 128: the two-launch form
    m.fused.use_raw_forward = False
    assert m.fused.raw_table(90) is None


@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("B", [1, 37, 4096])
def test_raw_forward_equals_pack_forward(g1, B, train):
    """The pack-free forward (records from the parameters, h of the workgroup's rows on the matrix cores) against the
    two-launch form (pack + fold, projection on x with Wc): the same sums in a different association -- loss within
    2e-6 relative, gradients within rtol 1e-4 -- and the same dropout stream."""
    gen = torch.Generator().manual_seed(B + 1)
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn(B, 30, 3, generator=gen).to(DEV)
    m = _model(FC_SMALL_CFG, golden_sd(g1), train=train)
    res = []
    for raw in (True, False):
        m.fused.use_raw_forward = raw
        res.append(_grads(m, y, traj, True, 4321))
    (v1, g1_, w1, b1, r1), (v0, g0, w0, b0, r0) = res
    assert r1 == r0
    assert abs(v1[0].item() - v0[0].item()) <= 2e-6 * abs(v0[0].item()) + 1e-6
    for a, b, what in ((g1_, g0, "stack"), (w1, w0, "feature W"), (b1, b0, "feature b")):
        ok, err = close(a.cpu(), b.cpu(), rtol=1e-4, floor=1e-5)
        assert ok, (what, err)


@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("B", [64, 4096])
def test_raw_forward_after_unfused_forward(B, train):
    """The smoke's sequence (random init, an unfused training forward, then the fused NLL): the unfused launches leave
    non-finite values in LDS, and the pack-free forward's h GEMM reads Wf's K padding (columns 90 .. 95 of FC_small)
    from LDS -- staged as zeros, so the loss stays finite and equals the two-launch form (parity unpinned beyond
    that: random init, no reference fixture)."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(FC_SMALL_CFG)
    del cfg["feature_networks"][1]["kwargs"]["dropout"]
    gen = torch.Generator().manual_seed(1)
    y = torch.randn(B, 19, generator=gen).to(DEV)
    traj = torch.randn(B, 30, 3, generator=gen).to(DEV)
    res = []
    for raw in (True, False):
        torch.manual_seed(2024_03_25)
        m = CondRealNVP_v2.from_config(cfg).to(DEV).train()
        m.fused.set_seed(3)
        with torch.no_grad():
            m(y, traj, log_det_J=True)
        m.fused.use_raw_forward = raw
        m.train(train)
        from bcnf_amd import _native as N
        N.check(N.lib().bcnf_lds_fill(ctypes.c_float(float("nan")), N.stream_handle(y.device)),
                "bcnf_lds_fill")                 # the residue the smoke met, made certain
        res.append(m.nll_loss(y, traj)[0].item())
    assert math.isfinite(res[0]) and abs(res[0] - res[1]) <= 2e-6 * abs(res[1]) + 1e-6, res


@pytest.mark.parametrize("nb", [2, 3])
def test_raw_forward_few_blocks(nb):
    """nb = 2 (both records prepared before the first barrier; the last block's record through rec_f) and 3."""
    cfg = _cfg((30, 3), 80, nb)
    m = _model(cfg, train=True, seed=5)
    assert m.fused.raw_table(90) is not None
    gen = torch.Generator().manual_seed(3)
    y = torch.randn(100, 19, generator=gen).to(DEV)
    traj = torch.randn(100, 30, 3, generator=gen).to(DEV)
    res = []
    for raw in (True, False):
        m.fused.use_raw_forward = raw
        res.append(_grads(m, y, traj, True, 77))
    (v1, g1_, w1, b1, _), (v0, g0, w0, b0, _) = res
    assert abs(v1[0].item() - v0[0].item()) <= 2e-6 * abs(v0[0].item()) + 1e-6
    for a, b, what in ((g1_, g0, "stack"), (w1, w0, "feature W"), (b1, b0, "feature b")):
        ok, err = close(a.cpu(), b.cpu(), rtol=1e-4, floor=1e-5)
        assert ok, (what, err)

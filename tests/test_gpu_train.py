"""GPU tests of the training-step kernels: fused NLL forward/backward, FusedAdam + clip, the feature-net
Linear GEMMs, and the HIP-graph TrainStep.

Numerics: each HIP kernel is compared with a plain PyTorch fp32 reference of the same op on the CPU
(torch.optim.Adam, torch.nn.utils.clip_grad_norm_, torch.nn.functional.linear) and the fused training
step with the reference's own golden fixture (tests/golden/g1_fc_small.npz: loss, Adam step + clip).
Tolerances are written per test.
"""
import numpy as np
import pytest
import torch

from conftest import FC_SMALL_CFG, close, golden_sd

pytestmark = pytest.mark.gpu

DEV = "cuda"


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def fresh_model(g1=None, train=False, seed=0):
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(seed)
    m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
    if g1 is not None:
        m.load_state_dict(golden_sd(g1))
    m.to(DEV)
    m.train(train)
    return m


# ---------------------------------------------------------------------------------------------- Adam
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adam_matches_torch_adam(wd):
    """Three steps over an odd-sized multi-tensor list; rtol 2e-6 / atol 1e-7 vs torch.optim.Adam (CPU fp32)."""
    from bcnf_amd.optim import FusedAdam
    gen = torch.Generator().manual_seed(3)
    shapes = [(109786,), (80, 90), (80,), (7,), (1, 1)]
    ref = [torch.randn(s, generator=gen).requires_grad_() for s in shapes]
    ours = [p.detach().clone().to(DEV).requires_grad_() for p in ref]
    opt_r = torch.optim.Adam(ref, lr=2e-3, weight_decay=wd)
    opt_o = FusedAdam(ours, lr=2e-3, weight_decay=wd)
    for _ in range(3):
        grads = [torch.randn(s, generator=gen) for s in shapes]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        for p, g in zip(ours, grads):
            p.grad = g.to(DEV)
        opt_r.step()
        opt_o.step()
    for a, b in zip(ours, ref):
        err = (a.detach().cpu() - b.detach()).abs().max().item()
        assert torch.allclose(a.detach().cpu(), b.detach(), rtol=2e-6, atol=1e-7), err
        sa = opt_o.state[a]
        sb = opt_r.state[b]
        # moments: ulp-level differences where m + (1-b1)(g-m) cancels (fma contraction) -> atol at
        # 1e-6 of the moment's scale
        for key in ("exp_avg", "exp_avg_sq"):
            ref_m = sb[key]
            assert torch.allclose(sa[key].cpu(), ref_m, rtol=1e-6, atol=1e-6 * ref_m.abs().max().item()), key
    assert float(opt_o.state[ours[0]]["step"]) == 3.0


def test_clip_after_step_matches_torch():
    """clip_grad_norm_ (max_norm 1) after the step: total norm rtol 1e-6, clipped grads rtol 1e-6."""
    from bcnf_amd.optim import FusedAdam, clip_grad_norm_
    gen = torch.Generator().manual_seed(5)
    shapes = [(109786,), (80, 90), (80,)]
    ref = [torch.randn(s, generator=gen).requires_grad_() for s in shapes]
    ours = [p.detach().clone().to(DEV).requires_grad_() for p in ref]
    grads = [torch.randn(s, generator=gen) for s in shapes]
    for p, g in zip(ref, grads):
        p.grad = g.clone()
    for p, g in zip(ours, grads):
        p.grad = g.to(DEV)
    opt = FusedAdam(ours, lr=1e-3)
    opt.step()
    n_ours = opt.clip_grad_norm_after_step(1.0)
    n_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    assert abs(n_ours.item() - n_ref.item()) <= 1e-6 * n_ref.item()
    for a, b in zip(ours, ref):
        assert torch.allclose(a.grad.cpu(), b.grad, rtol=1e-6, atol=1e-9)
    # standalone clip (no preceding step) on grads with norm < max_norm: coefficient 1, grads unchanged
    small = [torch.full((1000,), 1e-3, device=DEV).requires_grad_()]
    small[0].grad = torch.full((1000,), 1e-3, device=DEV)
    n = clip_grad_norm_(small, 1.0)
    assert abs(n.item() - (1000 * 1e-6) ** 0.5) < 1e-7
    assert torch.equal(small[0].grad, torch.full((1000,), 1e-3, device=DEV))


# --------------------------------------------------------------------------------------------- Linear
@pytest.mark.parametrize("rows,k,n", [(4096, 90, 80), (17, 5, 3), (1000, 33, 130), (1, 90, 80), (300, 16, 16)])
def test_linear_matches_torch(rows, k, n):
    """HIPLinear forward / dx / dW / db vs torch fp64 on CPU: |err| <= 1e-5 * (1 + max|ref|)."""
    from bcnf_amd.feature_network import HIPLinear
    gen = torch.Generator().manual_seed(rows + k + n)
    lin = HIPLinear(k, n)
    x = torch.randn(rows, k, generator=gen)
    dy = torch.randn(rows, n, generator=gen)
    xr = x.double().requires_grad_()
    wr = lin.weight.detach().double().requires_grad_()
    br = lin.bias.detach().double().requires_grad_()
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy.double())
    lin = lin.to(DEV)
    xg = x.to(DEV).requires_grad_()
    yg = lin(xg)
    yg.backward(dy.to(DEV))
    for got, ref in [(yg, yr), (xg.grad, xr.grad), (lin.weight.grad, wr.grad), (lin.bias.grad, br.grad)]:
        err = (got.detach().double().cpu() - ref.detach()).abs().max().item()
        assert err <= 1e-5 * (1.0 + ref.abs().max().item()), err


# ------------------------------------------------------------------------------------------ fused NLL
def test_nll_loss_matches_reference_golden(g1):
    """model.nll_loss (one fused launch) = the reference's loss; its backward = the reference's grads."""
    m = fresh_model(g1)
    flat = m.flat_parameters()
    vals = m.nll_loss(t(g1["y"]), t(g1["traj"]))
    loss = float(g1["loss"])
    v = vals.detach().cpu()
    assert abs(v[0].item() - loss) <= 1e-5 * abs(loss) + 1e-5
    assert v[0].item() == v[1].item() and v[2].item() == 0.0
    torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    named = dict(m.named_parameters())
    fp = m.fused
    g = flat[0].grad.cpu()
    n = 0
    for (off, k), p in zip(fp._offsets, fp.trainable):
        name = [kk for kk, vv in named.items() if vv is p][0]
        ok, err = close(g[off:off + k].view(p.shape), g1["grad/" + name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
        n += 1
    for name in ["feature_network_stack.feature_networks.1.nn.0.weight",
                 "feature_network_stack.feature_networks.1.nn.0.bias"]:
        ok, err = close(named[name].grad.cpu(), g1["grad/" + name], rtol=1e-4, floor=1e-4)
        assert ok, (name, err)
    assert n == 574


def test_nll_loss_equals_unfused_path_with_dropout(g1):
    """Training mode (dropout on): fused loss and gradient == forward + inn_nll_loss + autograd with the
    same RNG stream (rtol 1e-6 on the loss, 1e-5 on gradients); the fused kernel advances the offset."""
    from bcnf_amd import inn_nll_loss
    y, traj = t(g1["y"]), t(g1["traj"])
    m = fresh_model(g1, train=True)
    m.flat_parameters()
    m.fold_features = False        # the fused NLL kernel itself; the folded feature Linear: test_gpu_fold.py
    m.fused.set_seed(1234)
    vals = m.nll_loss(y, traj)
    torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    g_fused = m.fused.flat_param.grad.clone()
    gw_fused = m.feature_network_stack.feature_networks[1].nn[0].weight.grad.clone()
    assert int(m.fused.rng_state()[1].item()) == 1
    m.zero_grad(set_to_none=True)
    m.fused.flat_param.grad = None
    m.fused.set_seed(1234)
    z = m(y, traj, log_det_J=True)
    loss = inn_nll_loss(z, m.log_det_J)
    loss.backward()
    assert abs(loss.item() - vals[0].item()) <= 1e-6 * abs(loss.item())
    assert torch.allclose(m.fused.flat_param.grad, g_fused, rtol=1e-5, atol=1e-6)
    assert torch.allclose(m.feature_network_stack.feature_networks[1].nn[0].weight.grad, gw_fused,
                          rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------------------------------ TrainStep
def test_trainstep_matches_reference_step(g1):
    """One TrainStep (fused loss + FusedAdam + clip after step, eager) == the reference's Adam step."""
    from bcnf_amd.train import TrainStep
    m = fresh_model(g1)
    step = TrainStep(m, lr=2e-4, capture=False)
    loss, nll, mse = step.step(t(g1["y"]), t(g1["traj"]))
    ref = float(g1["loss"])
    assert abs(loss - ref) <= 1e-5 * abs(ref) + 1e-5 and nll == loss and mse == 0.0
    named = dict(m.named_parameters())
    n = 0
    for k in g1.keys():
        if k.startswith("after/"):
            ok, err = close(named[k[6:]].detach().cpu(), g1[k], rtol=1e-5, floor=1e-5)
            assert ok, (k, err)
            n += 1
    assert n > 500


def test_trainstep_graph_replay_equals_eager(g1):
    """HIP-graph TrainStep (with captured gather) == eager TrainStep over 3 dropout steps, bit for bit;
    the first step() applies exactly one update."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(11)
    pool_y = torch.randn(512, 19, generator=gen).to(DEV)
    pool_t = torch.randn(512, 30, 3, generator=gen).to(DEV)
    idxs = [torch.randperm(512, generator=gen)[:256].to(DEV) for _ in range(3)]
    res = []
    for capture, epoch in ((False, False), (True, False), (True, True)):
        m = fresh_model(g1, train=True)
        m.fused.set_seed(77)
        st = TrainStep(m, lr=2e-4, capture=capture)
        st.set_pool(pool_y, pool_t)
        if epoch:    # device-resident order + device cursor: no per-step index traffic
            st.set_epoch(torch.cat(idxs), 256)
            losses = [st.step_epoch() for _ in idxs]
        else:
            losses = [st.step_indexed(i) for i in idxs]
        res.append((losses, [p.detach().clone() for p in m.parameters()], int(m.fused.rng_state()[1].item())))
    (l0, p0, r0) = res[0]
    for (l1, p1, r1) in res[1:]:
        assert l0 == l1
        assert r0 == r1 == 3
        for a, b in zip(p0, p1):
            assert torch.equal(a, b)


def _epoch_pool(gen, n=768, blow_up=None):
    y = torch.randn(n, 19, generator=gen)
    traj = torch.randn(n, 30, 3, generator=gen)
    if blow_up is not None:            # rows whose NLL is ~1e8: the Trainer's divergence condition
        y[blow_up] *= 1e4
    return y.to(DEV), traj.to(DEV)


@pytest.mark.parametrize("unroll,batch", [(8, 192), (2, 192), (3, 192), (8, 48)])
def test_run_epoch_equals_per_step_loop(g1, unroll, batch):
    """run_epoch (back-to-back replays, one sync; `unroll` steps per captured graph, the remainder in unroll / 2,
    / 4 ... step graphs) == step_epoch per step: same logged values, parameters, Adam state, RNG offset, cursor and
    .grad (the last step's), bit for bit. Batch 48: 16 steps, run as 1 + (8 + 4 + 2 + 1)."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(21)
    py, pt = _epoch_pool(gen)
    nb = 768 // batch
    order = torch.randperm(768, generator=gen)[:nb * batch].to(DEV)
    res = []
    for batched in (False, True):
        m = fresh_model(g1, train=True)
        m.fused.set_seed(5)
        st = TrainStep(m, lr=2e-4)
        st.epoch_unroll = unroll
        st.set_pool(py, pt)
        st.set_epoch(order, batch)
        if batched:
            vals = st.run_epoch(1) + st.run_epoch()          # a partial run, then the rest of the epoch
        else:
            vals = [st.step_epoch() for _ in range(nb)]
        state = [v.clone() for s in st.opt.state.values() for v in s.values()]
        res.append((vals, [p.detach().clone() for p in m.parameters()], state,
                    m.fused.rng_state().clone(), st._epoch[1].item(), [p.grad.clone() for p in st.params]))
    (v0, p0, s0, r0, c0, g0), (v1, p1, s1, r1, c1, gr1) = res
    assert v0 == v1 and len(v1) == nb
    assert c0 == c1 == 0 and torch.equal(r0, r1)
    names = [f"param{i}" for i in range(len(p0))] + [f"state{i}" for i in range(len(s0))] + \
        [f"grad{i}" for i in range(len(g0))]
    for n, a, b in zip(names, p0 + s0 + g0, p1 + s1 + gr1):
        assert torch.equal(a, b), (n, float((a.float() - b.float()).abs().max()))


def test_run_epoch_divergence_halts_like_the_trainer(g1):
    """A batch with loss > 1e5 under check_divergence: run_epoch raises TrainingDivergedError and leaves
    parameters, Adam state, step count, RNG offset and cursor exactly as after that step (the reference
    raises right after the update of the diverged batch, trainer.py:166-169); later steps are no-ops."""
    from bcnf_amd.train import TrainStep, TrainingDivergedError
    gen = torch.Generator().manual_seed(22)
    order = torch.randperm(768, generator=gen)[:5 * 128]
    bad = order[2 * 128:3 * 128]                              # batch 2 diverges
    py, pt = _epoch_pool(gen, blow_up=bad)
    order = order.to(DEV)
    res = []
    for mode in ("per_step", "epoch", "eager_epoch"):
        m = fresh_model(g1, train=True)
        m.fused.set_seed(9)
        st = TrainStep(m, lr=2e-4, capture=mode != "eager_epoch")
        st.epoch_unroll = 2                                   # the halt lands inside a multi-step graph
        st.set_pool(py, pt)
        st.set_epoch(order, 128)
        if mode == "per_step":
            vals = [st.step_epoch() for _ in range(3)]
            assert vals[2][0] > 1e5 and all(v[0] < 1e5 for v in vals[:2])
        else:
            # eager_epoch: the per-step host check raises right after batch 2's update, before batch 3 runs
            with pytest.raises(TrainingDivergedError, match="at batch 2"):
                st.run_epoch(check_divergence=True)
            assert st._host_cursor == 3
        state = [v.clone() for s in st.opt.state.values() for v in s.values()]
        res.append(([p.detach().clone() for p in m.parameters()], state, m.fused.rng_state().clone(),
                    st._epoch[1].item()))
    (p0, s0, r0, c0) = res[0]
    for (p1, s1, r1, c1) in res[1:]:
        assert c0 == c1 == 3 and torch.equal(r0, r1)
        for a, b in zip(p0 + s0, p1 + s1):
            assert torch.equal(a, b)
        assert float(s1[0]) == 3.0                           # Adam step count: three updates applied


def test_captured_step_with_ragged_batches_equals_eager(g1):
    """The DataLoader's last batch is smaller (drop_last=False, trainer_data_handler.py:146): a captured TrainStep
    given batches of 128, 128, 1, 127, 128 samples runs the odd sizes eagerly and matches an eager TrainStep bit for
    bit (logged values and parameters); the 1-sample batch is not broadcast into the captured buffers."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(31)
    sizes = [128, 128, 1, 127, 128]
    batches = [(torch.randn(n, 19, generator=gen).to(DEV), torch.randn(n, 30, 3, generator=gen).to(DEV))
               for n in sizes]
    res = []
    for capture in (False, True):
        m = fresh_model(g1, train=True)
        m.fused.set_seed(41)
        st = TrainStep(m, lr=2e-4, capture=capture)
        vals = [st.step(y, tr) for y, tr in batches]
        res.append((vals, [p.detach().clone() for p in m.parameters()], [p.grad.clone() for p in st.params]))
    (v0, p0, g0), (v1, p1, g1_) = res
    assert v0 == v1
    for a, b in zip(p0 + g0, p1 + g1_):
        assert torch.equal(a, b)


def test_epoch_with_ragged_remainder_equals_eager_loop(g1):
    """An epoch order walked by run_epoch, then the epoch's ragged remainders (1 and 7 samples) through
    step_indexed, then run_epoch again == an eager TrainStep fed the same batches one by one: the remainders run
    eagerly without advancing the device cursor or writing an epoch history row (logged values, parameters, RNG
    offset and cursor bit for bit)."""
    from bcnf_amd.train import TrainStep
    gen = torch.Generator().manual_seed(23)
    py, pt = _epoch_pool(gen)
    perm = torch.randperm(768, generator=gen)
    order, rem1, rem7 = perm[:4 * 128].to(DEV), perm[600:601].to(DEV), perm[601:608]
    res = []
    for epoch in (False, True):
        m = fresh_model(g1, train=True)
        m.fused.set_seed(13)
        st = TrainStep(m, lr=2e-4, capture=epoch)
        st.set_pool(py, pt)
        batches = list(order.view(4, 128))
        if epoch:
            st.set_epoch(order, 128)
            vals = st.run_epoch()
            vals += [st.step_indexed(rem1), st.step_indexed(rem7)]     # rem7 from the host: checked there
            vals += st.run_epoch()
            cursor = st._epoch[1].item()
        else:
            vals = [st.step_indexed(b) for b in batches + [rem1, rem7] + batches]
            cursor = 0
        res.append((vals, [p.detach().clone() for p in m.parameters()], m.fused.rng_state().clone(), cursor))
    (v0, p0, r0, c0), (v1, p1, r1, c1) = res
    assert len(v1) == 10 and v0 == v1
    assert c0 == c1 == 0 and torch.equal(r0, r1)
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)


def test_step_indexed_rejects_out_of_range_indices(g1):
    from bcnf_amd.train import TrainStep
    m = fresh_model(g1, train=True)
    st = TrainStep(m, lr=2e-4)
    gen = torch.Generator().manual_seed(3)
    st.set_pool(torch.randn(64, 19, generator=gen).to(DEV), torch.randn(64, 30, 3, generator=gen).to(DEV))
    with pytest.raises(IndexError):
        st.step_indexed(torch.tensor([0, 5, 64], device=DEV))
    with pytest.raises(IndexError):
        st.set_epoch(torch.tensor([0, -1], device=DEV), 2)


def test_clip_grad_norm_over_more_tensors_than_one_launch_matches_torch():
    """bcnf_amd.optim.clip_grad_norm_ over 120 tensors (> BCNF_MAX_TENSORS = 48: the layerwise AnyGLU TrainStep's
    case) == torch.nn.utils.clip_grad_norm_ (norm and scaled gradients within 1e-6 relative)."""
    from bcnf_amd.optim import clip_grad_norm_
    g = torch.Generator().manual_seed(3)
    sizes = [37, 5000, 1] * 40
    ours = [torch.nn.Parameter(torch.zeros(n, device="cuda")) for n in sizes]
    ref = [torch.nn.Parameter(torch.zeros(n, device="cuda")) for n in sizes]
    for a, b, n in zip(ours, ref, sizes):
        gr = torch.randn(n, generator=g).to("cuda")
        a.grad, b.grad = gr.clone(), gr.clone()
    n_ours = clip_grad_norm_(ours, 1.0)
    n_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    assert abs(n_ours.item() - n_ref.item()) <= 1e-6 * n_ref.item()
    for a, b in zip(ours, ref):
        assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-9)


def test_clip_after_step_over_a_pre_reduced_partial_set_matches_fp64():
    """A 5.3M-parameter set (> CLIP_DIRECT_PARTIALS workgroup partials: k_sum_partials pre-reduces them, one
    1024-thread workgroup) plus ragged tensors: clip-after-step norm and scaled grads against the fp64 clip
    (torch.nn.utils.clip_grad_norm_'s formula) within 1e-5 relative. fp64, not torch's fp32 CPU norm: at 5.3M terms
    that one's own rounding is ~1e-4 relative."""
    from bcnf_amd.optim import FusedAdam
    gen = torch.Generator().manual_seed(11)
    shapes = [(5_300_001,), (37, 3), (1,)]
    grads = [torch.randn(s, generator=gen) for s in shapes]
    ours = [torch.zeros(s, device=DEV).requires_grad_() for s in shapes]
    for q, g in zip(ours, grads):
        q.grad = g.to(DEV)
    opt = FusedAdam(ours, lr=1e-3)
    opt.step()
    n_ours = opt.clip_grad_norm_after_step(1.0)
    n_ref = float(sum((g.double() ** 2).sum() for g in grads)) ** 0.5
    coef = min(1.0 / (n_ref + 1e-6), 1.0)
    assert abs(n_ours.item() - n_ref) <= 1e-5 * n_ref
    for a, g in zip(ours, grads):
        assert torch.allclose(a.grad.cpu().double(), g.double() * coef, rtol=1e-5, atol=1e-12)

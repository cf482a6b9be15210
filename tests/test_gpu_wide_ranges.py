"""GPU tests of the range-split wide backward (bcnf_wide_fold_backward_range, WideStack.range_blocks): the folded
wide backward run as descending real-block ranges, each range's coupling-gradient slice handed to a callback right
after its launches (TrainStep.overlap_ranges all-reduces it there), must equal the one-call backward bit for bit
(per output element the same GEMM K order; the split-K partials of a range use its own dead G slots) and every
slice must be final when it is handed over. One-way (S = 1) and two_way (S = 2) stacks, ragged batch, dropout on
with the same Philox stream in both runs."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _cfg(two_way, nb=5):
    return {"global": {"parameter_selection": [str(i) for i in range(19)]},
            "model": {"kwargs": {"size": 19, "nested_sizes": [48] * 3, "n_conditions": 80, "n_blocks": nb,
                                 "dropout": 0.2, "act_norm": True, "two_way": two_way}},
            "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                 {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}


def _grads(m, y, traj, ranges=None):
    st = m.fused
    m.zero_grad(set_to_none=True)
    st.flat_param.grad = None
    st.set_seed(7)
    seen, bucket = [], None
    if ranges is not None:
        n = st.flat.numel()
        bucket = torch.full((n + 9,), float("nan"), device=DEV)
        st.grad_bucket = (bucket, 5)
        st.range_blocks = ranges
        st.on_range = lambda lo, hi: seen.append((lo, hi, bucket[lo:hi].clone()))
    try:
        vals = m.nll_loss(y, traj)
        torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    finally:
        st.grad_bucket = st.range_blocks = st.on_range = None
    lin = m.feature_network_stack.feature_networks[1].nn[0]
    out = [st.flat_param.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone(), vals.detach().clone()]
    return out, seen, bucket


@pytest.mark.parametrize("two_way", [False, True], ids=["one_way", "two_way"])
@pytest.mark.parametrize("ranges", [[(3, 5), (1, 3), (0, 1)], [(4, 5), (3, 4), (2, 3), (1, 2), (0, 1)], [(0, 5)]],
                         ids=["3_ranges", "per_block", "one_range"])
def test_range_backward_equals_one_call(two_way, ranges):
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.wide import WideStack
    torch.manual_seed(3)
    m = CondRealNVP_v2.from_config(_cfg(two_way)).to(DEV).train()
    m.flat_parameters()
    assert isinstance(m.fused, WideStack)
    g = torch.Generator().manual_seed(4)
    B = 77
    y = torch.randn(B, 19, generator=g).to(DEV)
    traj = torch.randn(B, 30, 3, generator=g).to(DEV)
    ref, _, _ = _grads(m, y, traj)
    got, seen, bucket = _grads(m, y, traj, ranges)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    st = m.fused
    assert [(lo, hi) for lo, hi, _ in seen] == [(5 + st.block_offset(a), 5 + st.block_offset(b)) for a, b in ranges]
    for lo, hi, snap in seen:            # final when handed over
        assert torch.equal(snap, bucket[lo:hi])
    assert seen[0][1] == 5 + st.flat.numel() and seen[-1][0] == 5        # the slices tile the coupling gradient
    assert all(seen[i][0] == seen[i + 1][1] for i in range(len(seen) - 1))
    assert torch.equal(bucket[5:5 + st.flat.numel()], ref[0])


def _cfg_deep(two_way):
    c = _cfg(two_way)
    c["feature_networks"][1]["kwargs"]["sizes"] = [90, 64, 80]     # a layer below the folded Linear: its backward
    return c                                                       # runs on the launch stream during phase 2


def _side_grads(m, y, traj, side):
    st = m.fused
    m.zero_grad(set_to_none=True)
    st.flat_param.grad = None
    st.set_seed(7)
    st.side_stream = side
    try:
        vals = m.nll_loss(y, traj)
        torch.autograd.backward(vals, torch.tensor([1.0, 0.0, 0.0], device=DEV))
    finally:
        st.side_stream = None
        st.join_side(st.flat_param)
    return [st.flat_param.grad.clone(), vals.detach().clone()] + \
        [p.grad.clone() for p in m.feature_network_stack.parameters()]


@pytest.mark.parametrize("two_way", [False, True], ids=["one_way", "two_way"])
@pytest.mark.parametrize("B", [77, 1024])
def test_side_stream_backward_equals_one_call(two_way, B):
    """bcnf_wide_fold_backward_phase: phase 1 (chain, dL/dx, Gx, [dWf | dbf]) on the launch stream, phase 2 (the
    coupling parameter gradients) on a side stream while the feature layer below the fold runs its backward: equal
    to the one-call backward bit for bit, and the side buffer is what autograd adopted as .grad."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.wide import WideStack
    torch.manual_seed(3)
    m = CondRealNVP_v2.from_config(_cfg_deep(two_way)).to(DEV).train()
    m.flat_parameters()
    assert isinstance(m.fused, WideStack)
    g = torch.Generator().manual_seed(4)
    y = torch.randn(B, 19, generator=g).to(DEV)
    traj = torch.randn(B, 30, 3, generator=g).to(DEV)
    ref = _side_grads(m, y, traj, None)
    side = torch.cuda.Stream()
    for _ in range(2):
        got = _side_grads(m, y, traj, side)
        torch.cuda.synchronize()
        assert len(got) == len(ref)
        for a, b in zip(ref, got):
            assert torch.equal(a, b)


def test_side_stream_trainstep_equals_single_stream(monkeypatch):
    """TrainStep (captured) with the side-stream parameter gradients (BCNF_WIDE_SIDE=1) vs without: identical parameters after
    three steps (the join precedes Adam in the graph)."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.train import TrainStep
    g = torch.Generator().manual_seed(5)
    y = torch.randn(256, 19, generator=g).to(DEV)
    traj = torch.randn(256, 30, 3, generator=g).to(DEV)
    out = []
    for side in ("1", "0"):
        monkeypatch.setenv("BCNF_WIDE_SIDE", side)
        torch.manual_seed(3)
        m = CondRealNVP_v2.from_config(_cfg_deep(True)).to(DEV).train()
        ts = TrainStep(m, capture=True)
        assert (ts._side is not None) == (side == "1")
        m.fused.set_seed(11)
        vals = [ts.step(y, traj) for _ in range(3)]
        torch.cuda.synchronize()
        out.append((vals, [p.detach().clone() for p in m.parameters()]))
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)


def _guarded_workspace(monkeypatch, st, guards):
    """WideStack workspaces with NaN canaries of 64K floats before and after (16-B aligned views): any write of the
    library outside the workspace it was given shows up as a changed canary."""
    orig = type(st)._workspace

    def ws(self, batch, save, dev):
        inner = orig(self, batch, save, dev)
        n, g = inner.numel(), 1 << 16
        buf = torch.full((n + 2 * g,), float("nan"), device=dev)
        guards.append(buf)
        return buf[g:g + n]

    monkeypatch.setattr(type(st), "_workspace", ws)


@pytest.mark.parametrize("B", [24, 33, 34, 35, 36, 38, 48, 77])
def test_fold_backward_g_region_boundaries(monkeypatch, B):
    """VERDICT r04 item 4 (the r04ze illegal address): the folded wide backward puts the feature side's split-K
    partials (dL/dx, [dWf | dbf]; need nv * B * Xp and nv * C * Xp floats) at the END of the G region (nv * NH * B * HP
    floats, dead once the chain has run) and the coupling parameter gradients' partials at its head. At this shape
    (nv 5, NH 3, HP 52, C 80, Xp 68: region 780 B floats, [dWf | dbf] needs 27,200) the need crosses the region's size
    between B = 34 and 35 (B = 35 leaves the head 100 floats; FC_large at B = 48 leaves it 40K of 3.29M), so these batches
    cover a tail that exceeds the region (must reserve nothing and run unsplit: a reservation of more than the region
    pointed BEFORE it, into the activation region the parameter gradients read), a tail that fills it exactly or
    nearly (the head partials get a region of ~0 floats) and the usual case. Checks: no write outside the workspace
    (NaN canaries), phase 1 + phase 2 on two streams == one call bit for bit, folded == unfolded (rtol 1e-4)."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.wide import WideStack
    torch.manual_seed(3)
    m = CondRealNVP_v2.from_config(_cfg_deep(False)).to(DEV).train()
    m.flat_parameters()
    st = m.fused
    assert isinstance(st, WideStack)
    guards = []
    _guarded_workspace(monkeypatch, st, guards)
    g = torch.Generator().manual_seed(B)
    y = torch.randn(B, 19, generator=g).to(DEV)
    traj = torch.randn(B, 30, 3, generator=g).to(DEV)
    one = _side_grads(m, y, traj, None)
    two = _side_grads(m, y, traj, torch.cuda.Stream())
    torch.cuda.synchronize()
    for a, b in zip(one, two):
        assert torch.equal(a, b)
    for buf in guards:
        gsz = 1 << 16
        assert torch.isnan(buf[:gsz]).all() and torch.isnan(buf[-gsz:]).all(), "write outside the workspace"
    # folded vs unfolded (no fold split-K at all) on the same dropout streams
    m.fold_features = False
    try:
        assert m._wide_fold(y, (traj,)) is None
        ref = _side_grads(m, y, traj, None)
    finally:
        del m.fold_features
    assert torch.allclose(one[1], ref[1], rtol=2e-6, atol=1e-5)                  # the loss values
    scale = max(1.0, ref[0].abs().max().item())
    assert (one[0] - ref[0]).abs().max().item() <= 1e-4 * scale, "coupling gradient"
    for a, b in zip(one[2:], ref[2:]):
        assert (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item()), "feature gradient"

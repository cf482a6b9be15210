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

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

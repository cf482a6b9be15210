"""FC_small's in-kernel dropout masks, bit for bit against the test-side restatement of the kernel's stream
(tests/dropout_ref.py: Philox4x32-10, keep iff u32 >= round(p 2^32)), and the keep rate against nn.Dropout's p
(cnf.py:82-83) -- including p = 1e-6, which round 5's 16-bit threshold ran as no dropout at all."""
import copy

import numpy as np
import pytest
import torch

from conftest import FC_SMALL_CFG
from dropout_ref import keep_bits

pytestmark = pytest.mark.gpu


def _sample_of(t):                      # bcnf_stack.hip sample_of: thread -> sample within the workgroup's 16
    return (t >> 6) + 4 * ((t >> 4) & 3)


@pytest.mark.parametrize("NH", [7, 8], ids=["nh7_shared_low_half", "nh8_second_draw"])
@pytest.mark.parametrize("p", [0.383, 1e-6, 0.5])
def test_forward_dropout_masks_follow_the_32bit_rule(p, NH):
    """NH = 7 (FC_small): the draw's eighth 16-bit half is the low half of every unit's u32; NH = 8: tied units take
    their low halves from a second draw (dropout_bits)."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(FC_SMALL_CFG)
    cfg["model"]["kwargs"]["dropout"] = p
    cfg["model"]["kwargs"]["nested_sizes"] = [16] * NH
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(cfg).to("cuda").train()
    st = m.fused
    st.set_seed(0x5EED12345678)
    B, nb = 4096, 32
    g = torch.Generator().manual_seed(3)
    y = torch.randn(B, 19, generator=g).cuda()
    h = torch.randn(B, 80, generator=g).cuda()
    seed, off = (int(v) for v in st.rng_state().tolist())
    with torch.no_grad():
        _, _, _, (ws, _) = st.launch_forward(y, h, True, save=True)
    torch.cuda.synchronize()
    # activation records [k][workgroup][4][256 threads][4] float4 parts -> per thread (masked activation, masked
    # GELU derivative) of hidden layers 1..NH: a dropped unit is exactly 0
    rec = ws[: nb * B * 16 * 16].view(nb, B // 16, 4, 256, 4).permute(0, 1, 3, 2, 4).reshape(nb, B // 16, 256, 16)
    got = (rec[..., 1:2 * NH:2] != 0).cpu().numpy()
    t = np.arange(256)
    sample = np.arange(B // 16)[:, None] * 16 + _sample_of(t)[None, :]
    bits = keep_bits(p, seed, off, sample[None], np.arange(nb)[:, None, None], (t & 15)[None, None, :], nu=NH)
    want = ((bits[..., None] >> np.arange(NH, dtype=np.uint32)) & 1).astype(bool)
    assert got.shape == want.shape
    assert np.array_equal(got, want), int((got != want).sum())
    n = want.size
    drops = n - int(want.sum())
    lam = float(np.float32(p)) * n
    assert abs(drops - lam) < 4 * np.sqrt(lam * (1 - p)) + 1, (drops, lam)
    if p < 2.0**-17:
        assert drops > 0          # the 16-bit rule's threshold was 0 here: no unit ever dropped

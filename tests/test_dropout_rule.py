"""CPU checks of the FC_small kernels' dropout rule as restated in tests/dropout_ref.py (the GPU kernels are checked
bit for bit against it in tests/test_gpu_dropout.py): Philox4x32-10 against the Random123 known-answer vectors, and
the keep rule's effective p equal to nn.Dropout's p (cnf.py:82-83) to 2^-32 at every p, including p < 2^-17, which
round 5's 16-bit rule ran as no dropout at all."""
import numpy as np
import pytest

from dropout_ref import keep_bits, philox4x32_10, thresh32


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, out):
    got = philox4x32_10(*ctr, *key)
    assert tuple(int(v) for v in got) == out


@pytest.mark.parametrize("p", [0.383, 0.244, 0.407, 1e-6, 3e-9, 0.5, 0.0])
def test_threshold_is_p_to_2_pow_32(p):
    t = thresh32(p)
    assert abs(t / 2**32 - float(np.float32(p))) <= 2.0**-33
    if p > 0:
        assert t > 0                                   # round 5: round(p 2^16) = 0 for p < 2^-17


def test_keep_rule_statistics():
    """7M units at p = 0.383 (7 units per draw, the eighth half the shared low half): the drop fraction within 4 sigma
    of p; at p = 1e-6 over 64M units of 8-unit draws the drops are Poisson(64) within 4 sigma (the second-draw tie
    path, high half == 0, decides every one of them)."""
    rng = np.random.default_rng(5)
    s = rng.integers(0, 2**40, size=1 << 20)
    b = keep_bits(0.383, 1234, 77, s, 3, 5)
    drop = 7 * b.size - int(np.unpackbits(b.view(np.uint8)).sum())
    n = 7 * b.size
    assert abs(drop / n - 0.383) < 4 * np.sqrt(0.383 * 0.617 / n)
    drops = 0
    for blk in range(8):
        b = keep_bits(1e-6, 99, 3, s, blk, 7, nu=8)
        drops += 8 * b.size - int(np.unpackbits(b.view(np.uint8)).sum())
    n = 8 * 8 * s.size
    lam = 1e-6 * n
    assert drops > 0 and abs(drops - lam) < 4 * np.sqrt(lam), (drops, lam)

"""Test-side restatement of the FC_small kernels' dropout draw (bcnf_device.h: philox4x32_10, dropout_bits), numpy.

Not the reference's RNG: the reference draws nn.Dropout masks with torch's generator (cnf.py:82-83), which no
in-kernel generator can reproduce, so training parity is statistical plus exact fused == unfused equality on one
stream. This module pins the kernel's own stream bit for bit: Philox4x32-10 (Salmon et al. 2011, checked
against the Random123 known-answer vectors in tests/test_dropout_rule.py) and the keep rule "u32 >= round(p 2^32)".
"""
import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_U32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint32-valued arrays (any broadcastable shapes); returns four uint64 arrays."""
    c0, c1, c2, c3, k0, k1 = (np.asarray(v, dtype=np.uint64) & _U32 for v in (c0, c1, c2, c3, k0, k1))
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _U32, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _U32
        k0 = (k0 + _W0) & _U32
        k1 = (k1 + _W1) & _U32
    return c0, c1, c2, c3


def thresh32(p):
    """round(p 2^32) of the float32 p the library stores (BcnfStackDesc.dropout), clamped to 2^32 - 1."""
    return int(min(4294967295.0, np.floor(float(np.float32(p)) * 4294967296.0 + 0.5)))


def _halves(r):
    out = []
    for w in r:
        out += [w & np.uint64(0xFFFF), w >> np.uint64(16)]
    return out                                        # the 8 16-bit halves in the kernel's unit order


def keep_bits(p, seed, offset, sample, block, lane, tag=0, nu=7):
    """uint32 array of keep bits per (sample, block, lane) (broadcast) for a stack of nu hidden layers, bit i = unit i
    (hidden layer i + 1): keep iff u_i >= thresh32(p), u_i = (high 16 bits: half i of the draw, low 16 bits: the draw's
    eighth half when nu < 8, else half i of a second draw with counter tag bit 29)."""
    seed, offset = int(seed) & (2**64 - 1), int(offset) & (2**64 - 1)
    sample = np.asarray(sample, dtype=np.int64).astype(np.uint64)
    block = np.asarray(block, dtype=np.uint64)
    lane = np.asarray(lane, dtype=np.uint64)
    c1 = ((sample >> np.uint64(32)) ^ (block << np.uint64(8)) ^ np.uint64(tag)) & _U32
    k0, k1 = seed & 0xFFFFFFFF, ((seed >> 32) ^ (offset >> 32)) & 0xFFFFFFFF
    hi = _halves(philox4x32_10(sample & _U32, c1, lane, offset & 0xFFFFFFFF, k0, k1))
    if nu < 8:
        lo = [hi[7]] * 8
    else:
        lo = _halves(philox4x32_10(sample & _U32, c1 ^ np.uint64(0x20000000), lane, offset & 0xFFFFFFFF, k0, k1))
    t = np.uint64(thresh32(p))
    bits = np.zeros(np.broadcast(sample, block, lane).shape, dtype=np.uint32)
    for i in range(nu):
        u = (hi[i] << np.uint64(16)) | lo[i]
        bits |= (u >= t).astype(np.uint32) << np.uint32(i)
    return bits

"""Synthetic ballistic batches (bcnf_amd/data.py) are finite and physically plausible."""
import numpy as np

from bcnf_amd.data import PARAMETERS, simulate


def test_simulate_finite_and_shaped():
    y, tr = simulate(4096, seed=3)
    assert y.shape == (4096, len(PARAMETERS)) == (4096, 19)
    assert tr.shape == (4096, 30, 3)           # len(arange(0, 2.0, 0.067)) == 30 (physics.py:144)
    assert np.isfinite(y).all() and np.isfinite(tr).all()
    assert np.allclose(tr[:, 0, :], y[:, :3], atol=1e-5)   # trajectories start at x0


def test_simulate_deterministic():
    a = simulate(64, seed=11)
    b = simulate(64, seed=11)
    assert all(np.array_equal(u, v) for u, v in zip(a, b))

"""Synthetic ballistic-trajectory batches: a vectorised restatement of the reference's
simulator so benchmarks run on realistic conditions without the offline-unavailable HF datasets.

* ODE: ballistic_ODE (src/bcnf/simulation/physics.py:7-50):
      dv/dt = g - g rho (4/3) pi r^3 / m - (0.5 b / m) (v^2 v/|v| - w^2 w/|w|) + a
  integrated with classical RK4 (16 sub-steps per frame) on the reference's time grid t = arange(0, T, dt)
  (physics.py:144),
  positions x_i = x_{i-1} + v_i dt (physics.py:150-152), no impact break (configs use break_on_impact False).
* Priors: configs/data/config.yaml (polar x0/v0/w in the xy-plane, gamma g / rho / r / Cd, m).
* y: the 19 parameters of trajectory_FC_small's `parameter_selection`, in that order.
"""
from __future__ import annotations

import numpy as np

PARAMETERS = ['x0_x', 'x0_y', 'x0_z', 'v0_x', 'v0_y', 'v0_z', 'g', 'w_x', 'w_y', 'w_z',
              'b', 'm', 'a_x', 'a_y', 'a_z', 'r', 'A', 'Cd', 'rho']


def _polar(rng, n, std):
    r = np.abs(rng.normal(0.0, std, n))
    phi = rng.uniform(0.0, 2.0 * np.pi, n)
    return r * np.cos(phi), r * np.sin(phi)


def _dvdt(v, g, w, b, m, rho, r, a):
    vn = np.linalg.norm(v, axis=1, keepdims=True)
    wn = np.linalg.norm(w, axis=1, keepdims=True)
    vn = np.where(vn == 0, 1.0, vn)
    wn = np.where(wn == 0, 1.0, wn)
    buoy = g * rho * (4.0 / 3.0) * (np.pi * r ** 3) / m
    drag = (0.5 * b / m) * (v ** 2 * v / vn - w ** 2 * w / wn)
    return g - buoy - drag + a


def simulate(n: int, seed: int = 2024_03_25, T: float = 2.0, dt: float = 0.067, substeps: int = 16):
    """Return (y (n, 19) float32, trajectories (n, len(arange(0,T,dt)), 3) float32)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x0x, x0y = _polar(rng, n, 20.0)
    x0z = rng.uniform(0.1, 2.5, n)
    v0x, v0y = _polar(rng, n, 15.0)
    v0z = rng.normal(7.0, 5.0, n)
    wx, wy = _polar(rng, n, 3.0)
    wz = rng.normal(0.0, 1.0, n)
    gz = -rng.gamma(9.81, 1.0, n)
    rho = rng.gamma(3.5, 0.35, n)
    r = rng.gamma(1.75, 0.05, n) + 1e-3
    cd = rng.gamma(2.0, 0.1, n)
    m = rng.gamma(2.0, 0.5, n) + 0.05
    A = np.pi * r ** 2
    b = 0.5 * rho * A * cd
    zeros = np.zeros(n)

    g = np.stack([zeros, zeros, gz], 1)
    w = np.stack([wx, wy, wz], 1)
    a = np.stack([zeros, zeros, zeros], 1)
    bb, mm, rr, rh = b[:, None], m[:, None], r[:, None], rho[:, None]

    t = np.arange(0.0, T, dt)
    steps = len(t)
    v = np.stack([v0x, v0y, v0z], 1)
    x = np.stack([x0x, x0y, x0z], 1)
    traj = np.empty((n, steps, 3))
    traj[:, 0] = x
    f = lambda vv: _dvdt(vv, g, w, bb, mm, rr, rh, a)  # noqa: E731
    for i in range(1, steps):
        h = (t[i] - t[i - 1]) / substeps     # odeint is adaptive; fixed RK4 needs sub-steps for
        for _ in range(substeps):            # the stiff light-and-draggy tail of the priors
            k1 = f(v)
            k2 = f(v + 0.5 * h * k1)
            k3 = f(v + 0.5 * h * k2)
            k4 = f(v + h * k3)
            v = v + (h / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        x = x + v * dt
        traj[:, i] = x
    y = np.stack([x0x, x0y, x0z, v0x, v0y, v0z, gz, wx, wy, wz, b, m, zeros, zeros, zeros, r, A, cd, rho], 1)
    return y.astype(np.float32), traj.astype(np.float32)


class DeviceBatches:
    """A device-resident pool of samples served as pre-shuffled batches (the Trainer's DataLoader
    shuffle without its per-sample Python collate: SURVEY §7 'Trainer overheads')."""

    def __init__(self, n_pool: int, batch: int, device, seed: int = 2024_03_25, normalize: bool = True):
        import torch
        y, traj = simulate(n_pool, seed)
        y_t = torch.from_numpy(y)
        tr_t = torch.from_numpy(traj)
        if normalize:   # standardise so the synthetic NLL stays in the reference's training regime
            y_t = (y_t - y_t.mean(0)) / (y_t.std(0) + 1e-6)
            tr_t = (tr_t - tr_t.mean((0, 1))) / (tr_t.std((0, 1)) + 1e-6)
        self.y = y_t.to(device)
        self.traj = tr_t.to(device)
        self.batch = batch
        self.n = n_pool
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self._perm = None
        self._pos = 0
        self.device = device

    def next_indices(self):
        import torch
        if self._perm is None or self._pos + self.batch > self.n:
            self._perm = torch.randperm(self.n, generator=self.gen).to(self.device)
            self._pos = 0
        idx = self._perm[self._pos:self._pos + self.batch]
        self._pos += self.batch
        return idx

"""CPU ORACLE for re-simulation — TEST INFRASTRUCTURE ONLY.

Only `tests/` and `bench.py`'s `cpu_baseline` leg may import this module, and only as the checker / CPU baseline.
The product path (`bcnf_amd.resimulation`) never imports it.

A restatement of the reference's algorithm with the reference's own integrator (scipy.integrate.odeint, LSODA at its
default tolerances; scipy 1.15.3 in this image):
  * ballistic_ODE           physics.py:7-50   dv/dt = g - g rho (4/3) pi r^3 / m - (0.5 b / m)(v^2 v/|v| - w^2 w/|w|) + a
  * physics_ODE_simulation  physics.py:53-160 odeint over t = arange(0, T, dt); x[i] = x[i-1] + v[i] dt; impact break
  * resimulate              resimulation.py:21-59 (y_hat given): per (trajectory i, draw j), parameters from the draw
                            (ParameterIndexMapping.dictify) and the trajectory's fixed data_dict values; the process
                            pool is replaced by a loop (same results, the tasks are independent)
Pinned against fixtures produced by running the reference itself (`tests/golden/make_golden.py` g14):
`tests/test_resim.py`.
"""
from __future__ import annotations

import numpy as np
from scipy.integrate import odeint

PHYSICS_PARAMETERS = ("x0_x", "x0_y", "x0_z", "v0_x", "v0_y", "v0_z", "g_x", "g_y", "g_z", "w_x", "w_y", "w_z",
                      "b", "m", "rho", "r", "a_x", "a_y", "a_z")


def ballistic_rhs(v, t, g, w, b, m, rho, r, a):
    """physics.py:42 (same expression, same elementwise v^2 v / |v| drag)."""
    return g - g * rho * (4 / 3) * (np.pi * r ** 3) / m - (0.5 * b / m) * (
        v ** 2 * v / np.linalg.norm(v) - w ** 2 * w / np.linalg.norm(w)) + a


def simulate(p: dict, T: float, dt: float, break_on_impact: bool) -> np.ndarray:
    """physics.py:137-160 for one parameter dict (the 19 PHYSICS_PARAMETERS, float64)."""
    x0 = np.array([p["x0_x"], p["x0_y"], p["x0_z"]], dtype=np.float64)
    v0 = np.array([p["v0_x"], p["v0_y"], p["v0_z"]], dtype=np.float64)
    g = np.array([p["g_x"], p["g_y"], p["g_z"]], dtype=np.float64)
    w = np.array([p["w_x"], p["w_y"], p["w_z"]], dtype=np.float64)
    a = np.array([p["a_x"], p["a_y"], p["a_z"]], dtype=np.float64)
    t = np.arange(0, T, dt)
    with np.errstate(all="ignore"):
        v = odeint(ballistic_rhs, v0, t, args=(g, w, float(p["b"]), float(p["m"]), float(p["rho"]), float(p["r"]), a))
        x = np.zeros((v.shape[0], 3))
        x[0] = x0
        for i in range(1, v.shape[0]):
            x[i] = x[i - 1] + v[i] * dt
            if x[i, 2] < 0 and break_on_impact:
                ti = -x[i - 1, 2] / v[i, 2]
                x[i] = x[i - 1] + v[i] * ti
                x[i:] = x[i]
                break
    return x


def resimulate(y_hat: np.ndarray, parameters: list[str], data_dict: dict, T: float, dt: float,
               break_on_impact: bool, traj=None) -> np.ndarray:
    """resimulation.py:40-59 with y_hat (M, N, D) given: (N, M, len(t), 3) float64. `traj` restricts the
    trajectories (bounded CPU-baseline samples)."""
    M, N = y_hat.shape[0], y_hat.shape[1]
    fixed_names = [k for k in data_dict if k not in parameters]
    out = []
    for i in (range(N) if traj is None else traj):
        fixed = {k: data_dict[k][i] for k in fixed_names if k in PHYSICS_PARAMETERS}
        rows = []
        for j in range(M):
            p = {name: y_hat[j, i, c] for c, name in enumerate(parameters) if name in PHYSICS_PARAMETERS}
            p.update(fixed)
            rows.append(simulate({k: float(v) for k, v in p.items()}, T, dt, break_on_impact))
        out.append(rows)
    return np.array(out)

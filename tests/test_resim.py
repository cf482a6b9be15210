"""Re-simulation (simulation/resimulation.py:21-59, physics.py:53-160).

CPU: the oracle (scipy odeint, the reference's own integrator) against the g14 fixtures the reference produced, the
host-side parameter mapping and its errors. GPU: `bcnf_resimulate` (adaptive Dormand-Prince 5(4) in fp64, one thread
per trajectory) against the fixtures and the oracle.

Tolerance: odeint (LSODA) controls its local error at rtol = atol = 1.49e-8 and the kernel at 1e-10, so the two
differ by odeint's global error on the velocities, summed into the positions over the grid; the reference also rounds
kd = 0.5 b / m and part of the buoyancy to float32 when the parameters are float32 draws. Positions (metres, |x| up
to ~100) are compared at rtol = atol = 2e-6.
"""
import os
import types
import warnings

import numpy as np
import pytest
import torch

from bcnf_amd.resimulation import (PHYSICS_PARAMETERS, STATUS_STEPS, _columns, _warn_unfinished, resimulate,
                                   resimulate_device, time_grid)
from bcnf_amd.utils import ParameterIndexMapping
from oracle import resim_oracle as RO

G14 = os.path.join(os.path.dirname(__file__), "golden", "g14_resim.npz")
RTOL = ATOL = 2e-6


def _g14():
    return np.load(G14)


GRIDS = {"a": (2.0, 1 / 15, False), "b": (2.0, 1 / 15, True), "c": (10.0, 0.1, False)}


def test_oracle_matches_reference_physics():
    d = _g14()
    P = d["params"]
    for tag, (T, dt, brk) in GRIDS.items():
        ref = d["x_" + tag]
        for k in range(P.shape[0]):
            x = RO.simulate(dict(zip(PHYSICS_PARAMETERS, P[k])), T, dt, brk)
            np.testing.assert_allclose(x, ref[k], rtol=1e-9, atol=1e-9, equal_nan=True, err_msg=f"{tag}[{k}]")
    assert np.isnan(d["x_a"][7, 1:]).all() and not np.isnan(d["x_a"][7, 0]).any()    # zero wind: NaN from t[1]


def _resim_inputs(d):
    names = [str(s) for s in d["names"]]
    fixed = d["fixed_phys"]
    N = fixed.shape[0]
    data_dict = {q: list(fixed[:, c]) for c, q in enumerate(PHYSICS_PARAMETERS)}
    data_dict.update(g=list(d["g_extra"]), A=list(d["A_extra"]), Cd=[0.2] * N,
                     trajectories=[np.zeros((30, 3)) for _ in range(N)])
    return names, data_dict


def test_oracle_matches_reference_resimulate():
    d = _g14()
    names, data_dict = _resim_inputs(d)
    x = RO.resimulate(d["y_hat"], names, data_dict, 2, 1 / 15, True)
    assert x.shape == d["resim"].shape == (5, 6, 30, 3)
    np.testing.assert_allclose(x, d["resim"], rtol=RTOL, atol=ATOL)


def test_parameter_mapping_and_errors():
    names = ["x0_x", "x0_y", "x0_z", "v0_x", "v0_y", "v0_z", "g", "w_x", "w_y", "w_z", "b", "m", "a_x", "a_y",
             "a_z", "r", "A", "Cd", "rho"]
    cols = _columns(names, ["g_x", "g_y", "g_z", "trajectories"])
    assert cols[:6] == [0, 1, 2, 3, 4, 5] and cols[6:9] == [-1, -1, -1]
    assert cols[12:16] == [10, 11, 18, 15] and cols[16:] == [12, 13, 14]
    with pytest.raises(TypeError, match="g_z"):
        _columns(names, ["g_x", "g_y"])
    with pytest.raises(TypeError, match="multiple values"):
        _columns(names, ["g_x", "g_y", "g_z", "dt"])
    assert len(time_grid(2, 1 / 15)) == 30 and len(time_grid(10, 0.1)) == 100


def test_no_cpu_path():
    y = torch.zeros(2, 3, 19)
    with pytest.raises(RuntimeError, match="HIP device only"):
        resimulate_device(y, 2, 1 / 15, {}, ParameterIndexMapping(list(PHYSICS_PARAMETERS)), device="cpu")


def test_unfinished_trajectories_warn():
    """resimulate() never returns a silent NaN row for a trajectory the integrator could not finish."""
    st = torch.zeros(3, 4, dtype=torch.int32)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert _warn_unfinished(st) == 0
        st[0, 1] = 1                                   # NONFINITE (zero wind): NaN in the reference as well
        assert _warn_unfinished(st) == 0
    st[2, 3] = STATUS_STEPS
    st[1, 0] = STATUS_STEPS
    with pytest.warns(RuntimeWarning, match="2 of 12 trajectories did not finish"):
        assert _warn_unfinished(st) == 2


# ---------------------------------------------------------------------------------------------------------- GPU
def _all_from_draws(P, dtype=torch.float64):
    """y_hat (1, n, 19) carrying every physics parameter, mapping = PHYSICS_PARAMETERS."""
    return torch.tensor(P, dtype=dtype).unsqueeze(0).cuda(), ParameterIndexMapping(list(PHYSICS_PARAMETERS))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_gpu_physics_vs_reference(tag):
    d = _g14()
    T, dt, brk = GRIDS[tag]
    y, pim = _all_from_draws(d["params"])
    x, att, st = resimulate_device(y, T, dt, {}, pim, break_on_impact=brk, return_status=True)
    x = x[:, 0].cpu().numpy()
    np.testing.assert_allclose(x, d["x_" + tag], rtol=RTOL, atol=ATOL, equal_nan=True)
    st = st.cpu().numpy()[:, 0]
    assert st[7] == 1 and (np.delete(st, 7) == 0).all()
    assert (att.cpu().numpy()[:, 0] > 0).sum() == 39


@pytest.mark.gpu
def test_gpu_resimulate_vs_reference():
    d = _g14()
    names, data_dict = _resim_inputs(d)
    model = types.SimpleNamespace(parameter_index_mapping=ParameterIndexMapping(names), device="cuda:0")
    x = resimulate(model, 2, 1 / 15, data_dict, d["y_hat"], break_on_impact=True, verbose=False)
    assert x.dtype == np.float64 and x.shape == (5, 6, 30, 3)
    np.testing.assert_allclose(x, d["resim"], rtol=RTOL, atol=ATOL)
    xd = resimulate(model, 2, 1 / 15, data_dict, torch.from_numpy(d["y_hat"]).cuda(), break_on_impact=True,
                    verbose=False)
    np.testing.assert_array_equal(x, xd)


@pytest.mark.gpu
@pytest.mark.parametrize("brk", [False, True])
def test_gpu_vs_oracle_random(brk):
    rng = np.random.Generator(np.random.PCG64(77))
    n = 96
    P = np.zeros((n, 19))
    for k in range(n):
        P[k] = [*(rng.normal(0, 15, 2)), rng.uniform(0.1, 2.5), *(rng.normal(0, 12, 2)), rng.normal(7, 5),
                0.0, 0.0, -rng.gamma(9.81, 1.0), *(rng.normal(0, 3, 3)), rng.gamma(2.0, 0.005), rng.gamma(2, 0.5) + 0.05,
                rng.gamma(3.5, 0.35), rng.gamma(1.75, 0.05) + 1e-3, *(rng.normal(0, 0.3, 3))]
    y, pim = _all_from_draws(P)
    x = resimulate_device(y, 2.0, 1 / 15, {}, pim, break_on_impact=brk)[:, 0].cpu().numpy()
    for k in range(0, n, 3):
        ref = RO.simulate(dict(zip(PHYSICS_PARAMETERS, P[k])), 2.0, 1 / 15, brk)
        np.testing.assert_allclose(x[k], ref, rtol=RTOL, atol=ATOL, err_msg=str(k))


@pytest.mark.gpu
def test_gpu_float32_draws_and_determinism():
    d = _g14()
    P = d["params"].astype(np.float32)
    y32, pim = _all_from_draws(P, torch.float32)
    y64 = y32.double()
    a = resimulate_device(y32, 2.0, 1 / 15, {}, pim, break_on_impact=True)
    b = resimulate_device(y64, 2.0, 1 / 15, {}, pim, break_on_impact=True)
    c = resimulate_device(y32, 2.0, 1 / 15, {}, pim, break_on_impact=True)
    assert torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(b, 7.0))
    assert torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(c, 7.0))
    # a trajectory's result does not depend on its position in the launch
    sub = resimulate_device(y32[:, 13:29], 2.0, 1 / 15, {}, pim, break_on_impact=True)
    assert torch.equal(torch.nan_to_num(sub, 7.0), torch.nan_to_num(a[13:29], 7.0))


@pytest.mark.gpu
def test_gpu_draw_major_layout_and_edges():
    d = _g14()
    P = d["params"][:6]
    # M = 3 draws of N = 2 trajectories: y_hat[j, i] -> x[i, j]
    y = torch.tensor(np.stack([P[0:2], P[2:4], P[4:6]]), dtype=torch.float64).cuda()
    pim = ParameterIndexMapping(list(PHYSICS_PARAMETERS))
    x = resimulate_device(y, 2.0, 1 / 15, {}, pim).cpu().numpy()
    assert x.shape == (2, 3, 30, 3)
    for j in range(3):
        for i in range(2):
            np.testing.assert_allclose(x[i, j], d["x_a"][2 * j + i], rtol=RTOL, atol=ATOL)
    one = resimulate_device(y, 0.05, 0.1, {}, pim).cpu().numpy()          # arange(0, 0.05, 0.1) = [0]: x0 only
    assert one.shape == (2, 3, 1, 3)
    np.testing.assert_array_equal(one[:, :, 0], y.permute(1, 0, 2)[:, :, :3].cpu().numpy())
    with pytest.raises(IndexError):
        resimulate_device(y, 0.0, 0.1, {}, pim)
    model = types.SimpleNamespace(parameter_index_mapping=pim, device="cuda:0")
    assert resimulate(model, 2, 1 / 15, {}, np.zeros((0, 4, 19)), verbose=False).shape == (4, 0)
    assert resimulate(model, 2, 1 / 15, {}, np.zeros((3, 0, 19)), verbose=False).shape == (0,)


@pytest.mark.gpu
def test_gpu_attempt_bound_reports_steps_status():
    """A trajectory stopped by the attempt bound is NaN from the first grid time it missed, with status STEPS."""
    d = _g14()
    y, pim = _all_from_draws(d["params"][:4])
    x, att, st = resimulate_device(y, 2.0, 1 / 15, {}, pim, max_attempts=5, return_status=True)
    st = st.cpu().numpy()[:, 0]
    assert (st == STATUS_STEPS).all() and (att.cpu().numpy() == 6).all()
    x = x.cpu().numpy()[:, 0]
    assert not np.isnan(x[:, 0]).any() and np.isnan(x[:, -1]).all()
    with pytest.warns(RuntimeWarning, match="4 of 4"):
        _warn_unfinished(torch.from_numpy(st))

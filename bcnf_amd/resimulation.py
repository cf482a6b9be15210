"""Re-simulation of posterior draws on the GPU (psaegert/bcnf src/bcnf/simulation/resimulation.py:21-59; SURVEY §8f-2:
"resimulate ... is the next bottleneck after that").

The reference samples y_hat (M draws x N trajectories x D) with `model.sample(..., outer=True)`, copies it to the
host and maps `resimulate_trajectory` (resimulation.py:12-18) over every (draw j, trajectory i) in a
ProcessPoolExecutor: one scipy `odeint` (LSODA) integration of the ballistic velocity ODE per task
(physics.py:53-160). Here the draws stay on the device and ONE launch of `bcnf_resimulate` (bcnf_amd/csrc/
bcnf_resim.hip) integrates all M * N trajectories, one fp64 thread each.

Same interface and semantics as the reference:
  * physics parameter q comes from the draw when the model predicts it (ParameterIndexMapping.dictify,
    resimulation.py:16) and from `data_dict[name][i]` otherwise (resimulation.py:53); a physics argument found in
    neither raises TypeError as the call would (physics.py:53-72 has no defaults for them);
  * t = np.arange(0, T, dt) (physics.py:141), x[0] = x0, x[s] = x[s-1] + v[s] dt, the impact break of physics.py:154-159;
  * the result is a float64 numpy array (N, M, len(t), 3) = np.array(X_resimulation_list) (resimulation.py:59).
`n_procs` has no meaning here (there is no process pool) and is accepted for signature compatibility.

Numerics: odeint solves the ODE to its default rtol = atol = 1.49e-8; the kernel's adaptive Dormand-Prince 5(4) runs
at 1e-10, so both approximate the same exact solution and differ by odeint's own error (tests/test_resim.py states
the tolerance). The reference builds its arrays from the draws' float32 scalars and mixes float32 / float64
arithmetic in ballistic_ODE; the kernel computes in float64 from the same float32 values.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native

# physics_ODE_simulation's parameters in signature order (physics.py:53-72)
PHYSICS_PARAMETERS = ("x0_x", "x0_y", "x0_z", "v0_x", "v0_y", "v0_z", "g_x", "g_y", "g_z", "w_x", "w_y", "w_z",
                      "b", "m", "rho", "r", "a_x", "a_y", "a_z")
_CALL_KEYWORDS = ("T", "dt", "break_on_impact")      # keywords resimulate_trajectory passes itself

STATUS_OK, STATUS_NONFINITE, STATUS_STEPS = 0, 1, 2   # include/bcnf_amd.h BCNF_RESIM_*


def time_grid(T: float, dt: float) -> np.ndarray:
    """t = np.arange(0, T, dt) exactly as physics.py:141 builds it."""
    return np.arange(0, T, dt)


def _columns(parameters: list[str], fixed_names: list[str]) -> list[int]:
    """Column of each physics parameter in the draw, -1 = a fixed (data_dict) value. Raises TypeError like the
    keyword call of resimulation.py:14-18 when a parameter is in neither, or a name collides with T / dt /
    break_on_impact."""
    pmap = {p: i for i, p in enumerate(parameters)}
    for name in list(parameters) + list(fixed_names):
        if name in _CALL_KEYWORDS:
            raise TypeError(f"physics_ODE_simulation() got multiple values for keyword argument '{name}'")
    cols = []
    for name in PHYSICS_PARAMETERS:
        if name in pmap:
            cols.append(pmap[name])
        elif name in fixed_names:
            cols.append(-1)
        else:
            raise TypeError(f"physics_ODE_simulation() missing 1 required positional argument: '{name}'")
    return cols


def resimulate_device(y_hat, T: float, dt: float, data_dict: dict, parameter_index_mapping,
                      break_on_impact: bool = False, rtol: float = 1e-10, atol: float = 1e-10,
                      max_attempts: int = 1_000_000, device=None, return_status: bool = False):
    """(N, M, len(t), 3) float64 positions on the device for draws y_hat (M, N, D) (torch tensor, any device, or
    numpy). With return_status, also (attempts, status) int32 (N, M): Dormand-Prince step attempts and BCNF_RESIM_*."""
    parameters = list(parameter_index_mapping.parameters)
    if device is None:
        device = y_hat.device if isinstance(y_hat, torch.Tensor) and y_hat.is_cuda else torch.device(
            "cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("bcnf_amd.resimulate runs on the HIP device only (no CPU path); got " + str(device))
    yt = torch.as_tensor(y_hat)
    if yt.ndim != 3:
        raise ValueError(f"y_hat must be (M, N, D), got shape {tuple(yt.shape)}")
    if yt.dtype not in (torch.float32, torch.float64):
        yt = yt.to(torch.float64)
    yt = yt.to(device).contiguous()
    M, N, D = yt.shape
    t = time_grid(T, dt)
    steps = len(t)
    fixed_names = [k for k in data_dict.keys() if k not in parameters]
    cols = _columns(parameters, fixed_names)
    if D < len(parameters) and any(c >= D for c in cols):
        raise IndexError(f"y_hat has {D} columns, the parameter mapping needs {max(cols) + 1}")
    if steps == 0:        # x_sol = zeros((0, 3)); x_sol[0] = x0 (physics.py:147-148)
        raise IndexError("index 0 is out of bounds for axis 0 with size 0")
    fixed = np.full((N, len(PHYSICS_PARAMETERS)), np.nan, dtype=np.float64)
    for q, name in enumerate(PHYSICS_PARAMETERS):
        if cols[q] < 0:
            vals = data_dict[name]
            fixed[:, q] = [float(vals[i]) for i in range(N)]
    x = torch.empty((N, M, steps, 3), dtype=torch.float64, device=device)
    attempts = torch.empty((N, M), dtype=torch.int32, device=device) if return_status else None
    status = torch.empty((N, M), dtype=torch.int32, device=device) if return_status else None
    if M * N:
        fixed_d = torch.from_numpy(fixed).to(device)
        tgrid_d = torch.from_numpy(np.ascontiguousarray(t, dtype=np.float64)).to(device)
        col_arr = (ctypes.c_int32 * len(cols))(*cols)
        L = _native.lib()
        with torch.cuda.device(device):
            _native.check(L.bcnf_resimulate(_native.ptr(yt), 1 if yt.dtype == torch.float64 else 0, M, N, D, col_arr,
                                            _native.ptr(fixed_d), _native.ptr(tgrid_d), steps, float(dt),
                                            1 if break_on_impact else 0, float(rtol), float(atol), int(max_attempts),
                                            _native.ptr(x), _native.ptr(attempts), _native.ptr(status),
                                            _native.stream_handle(device)), "bcnf_resimulate")
    if return_status:
        return x, attempts, status
    return x


def resimulate(model, T: int, dt: float, data_dict: dict[str, list], y_hat=None, *conditions: torch.Tensor,
               m_samples: int = 1000, break_on_impact: bool = False, n_procs: int | None = None,
               batch_size: int = 100, verbose: bool = True) -> np.ndarray:
    """resimulation.py:21-59 with the same arguments and result (float64 numpy (N, M, len(arange(0, T, dt)), 3))."""
    if y_hat is None:
        if len(conditions) != model.feature_network_stack.n_distinct_conditions:
            raise ValueError(f"Expected {model.feature_network_stack.n_distinct_conditions} conditions, "
                             f"got {len(conditions)}")
        # same draws as the reference's sample(...).cpu(): the z stream is the CPU generator's; they stay on the device
        y_hat = model.sample(m_samples, *conditions, batch_size=batch_size, verbose=verbose, outer=True,
                             output_device=model.device)
    N = y_hat.shape[1]
    M = y_hat.shape[0]
    if verbose:
        print(f"Resimulating {N} trajectories {M} times")
    if N == 0:
        return np.array([])
    if M == 0:
        return np.array([[] for _ in range(N)])
    device = model.device if torch.device(model.device).type == "cuda" else None
    x, _, status = resimulate_device(y_hat, T, dt, data_dict, model.parameter_index_mapping,
                                     break_on_impact=break_on_impact, device=device, return_status=True)
    _warn_unfinished(status)
    return x.cpu().numpy()


def _warn_unfinished(status) -> int:
    """A trajectory the explicit Dormand-Prince pair could not finish (step-size underflow or the attempt bound:
    a stiff or divergent draw) is NaN from the first grid time it missed. The reference's LSODA switches method
    and returns values there (odeint warns when it struggles), so these rows are never silent: one warning with
    their count. NONFINITE rows (a zero wind: 0/0 in the drag term) are NaN in the reference as well."""
    n = int((status == STATUS_STEPS).sum().item()) if status is not None and status.numel() else 0
    if n:
        import warnings
        warnings.warn(f"bcnf_amd.resimulate: {n} of {status.numel()} trajectories did not finish (stiff or divergent "
                      f"draws: step-size underflow or the attempt bound); their positions are NaN from the first grid "
                      f"time that was not reached (resimulate_device(..., return_status=True) names them)",
                      RuntimeWarning, stacklevel=3)
    return n


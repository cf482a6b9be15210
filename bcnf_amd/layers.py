"""Variant coupling layers of the reference (src/bcnf/models/layers.py:9-78), same constructor arguments, submodule
names and state_dict keys:

* `AnyGLU(input_size, output_size, activation="GELU")`: linear_value(x) * activation(linear_gate(x))
  (layers.py:9-31). Its two Linear layers run on the library's fp32 MFMA GEMMs (`HIPLinear`) on the GPU; a stack
  built from AnyGLU couplings runs layer by layer (bcnf_amd/cnf.py, "layerwise" path), not in a fused kernel.
* `FFTLayer` / `FFTEnrichLayer` (layers.py:34-57): [Re rfft(x), Im rfft(x)] with norm="forward", and x
  concatenated with it.
* `LinearFFTEnriched(input_size, output_size)` (layers.py:60-78): linear(cat(x, rfft(x).real, rfft(x).imag)).
  The rfft is a fixed linear map F (2 (n//2 + 1) x n), so the layer IS a Linear with the effective weight
  W_eff = W[:, :n] + W[:, n:] F -- a stack of LinearFFTEnriched couplings runs on the fused wide-MLP kernels with
  W_eff (bcnf_amd/fft_stack.py), and the gradient maps back as dW[:, :n] = G, dW[:, n:] = G F^T.
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch
from torch import nn

from bcnf_amd.feature_network import HIPLinear


def _activation(name: str, **kwargs: Any) -> nn.Module:
    if hasattr(nn, name):
        return getattr(nn, name)(**kwargs)
    raise NotImplementedError(f"Layer {name} not implemented")


class AnyGLU(nn.Module):
    """Generalized linear unit with any activation (layers.py:9-31)."""

    def __init__(self, input_size: int, output_size: int, activation: str = "GELU",
                 activation_kwargs: dict[str, Any] | None = None) -> None:
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.linear_gate = HIPLinear(self.input_size, self.output_size)
        self.linear_value = HIPLinear(self.input_size, self.output_size)
        self.activation = _activation(activation, **(activation_kwargs or {}))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.linear_value(x) * self.activation(self.linear_gate(x))


def rfft_matrix(n: int, dtype=torch.float32, device=None) -> torch.Tensor:
    """F (2 (n//2 + 1) x n) with F x = cat(Re rfft(x, norm="forward"), Im rfft(x, norm="forward")): rows k < K hold
    cos(2 pi k i / n) / n, rows K + k hold -sin(2 pi k i / n) / n (angles reduced exactly in integers, fp64)."""
    K = n // 2 + 1
    k = np.arange(K)[:, None]
    i = np.arange(n)[None, :]
    ang = 2.0 * np.pi * ((k * i) % n) / n
    F = np.concatenate([np.cos(ang), -np.sin(ang)], axis=0) / n
    return torch.from_numpy(F).to(dtype=dtype, device=device)


class FFTLayer(nn.Module):
    """[Re rfft(x), Im rfft(x)] along the last axis, norm="forward" (layers.py:34-46)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        f = torch.fft.rfft(input=x, dim=-1, norm="forward")
        return torch.cat((f.real, f.imag), dim=-1)


class FFTEnrichLayer(nn.Module):
    """x concatenated with its FFTLayer output (layers.py:49-57)."""

    def __init__(self) -> None:
        super().__init__()
        self.fft = FFTLayer()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.cat((x, self.fft(x)), dim=-1)


class LinearFFTEnriched(nn.Module):
    """Linear over the input enriched with its FFT (layers.py:60-78)."""

    def __init__(self, input_size: int, output_size: int) -> None:
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.fft_enrich = FFTEnrichLayer()
        self.linear = nn.Linear(input_size + 2 * (input_size // 2 + 1), output_size)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.linear(self.fft_enrich(x))


LAYERS = {"AnyGLU": AnyGLU, "LinearFFTEnriched": LinearFFTEnriched, "FFTLayer": FFTLayer,
          "FFTEnrichLayer": FFTEnrichLayer}

"""Conditioning (feature) networks — PyTorch-ROCm, as the north star prescribes.

Restated from the reference's behaviour (src/bcnf/models/feature_network.py); their output h
(B, n_conditions) is the input boundary of the HIP coupling stack and dL/dh comes back out of it.

* FeatureNetworkStack          feature_network.py:28-73  (consumes one condition per ConcatenateCondition)
* ConcatenateCondition         feature_network.py:76-88
* FullyConnectedFeatureNetwork feature_network.py:114-145 (x.view(B,-1); Linear/[BN]/act/[Dropout] ...)
* LSTMFeatureNetwork           feature_network.py:148-178 — reference pools over dim 0 (the BATCH axis
  of a batch_first LSTM), which crashes for batch != seq_len. `pool_dim=0` keeps that
  behaviour bit-for-bit; `pool_dim=1` pools over time (documented fix used for trajectory_LSTM_large).
"""
from __future__ import annotations

from typing import Any, Type

import torch
from torch import nn


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b on the HIP GEMM kernels (bcnf_linear_forward / bcnf_linear_backward)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from bcnf_amd import _native as N
        rows, k = x.shape
        n = weight.shape[0]
        y = torch.empty((rows, n), dtype=torch.float32, device=x.device)
        N.check(N.lib().bcnf_linear_forward(N.ptr(x), N.ptr(weight), N.ptr(bias), rows, k, n, N.ptr(y),
                                            N.stream_handle(x.device)), "bcnf_linear_forward")
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from bcnf_amd import _native as N
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        rows, k = x.shape
        n = weight.shape[0]
        need_x, need_w, need_b = ctx.needs_input_grad
        dx = torch.empty_like(x) if need_x else None
        dw = torch.empty_like(weight) if (need_w or need_b) else None
        db = torch.empty(n, dtype=torch.float32, device=x.device) if (need_b and ctx.has_bias) else None
        work = None
        if dw is not None:
            wb = int(N.lib().bcnf_linear_work_bytes(rows, k, n))
            work = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=x.device)
        N.check(N.lib().bcnf_linear_backward(N.ptr(x), N.ptr(weight), N.ptr(dy), rows, k, n, N.ptr(dx), N.ptr(dw),
                                             N.ptr(db), N.ptr(work), N.stream_handle(x.device)),
                "bcnf_linear_backward")
        return dx, (dw if need_w else None), db


class HIPLinear(nn.Linear):
    """nn.Linear (same parameters / state_dict keys) whose fp32 GPU forward and backward run on the
    library's MFMA GEMM kernels; other devices / dtypes use torch's own linear."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and self.weight.dtype == torch.float32:
            return _LinearFn.apply(x.contiguous(), self.weight, self.bias)
        return super().forward(x)


class FeatureNetwork(nn.Module):
    input_size: int
    output_size: int

    @property
    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError


class ConcatenateCondition(FeatureNetwork):
    def __init__(self, input_size: int | None, output_size: int, dim: int = -1) -> None:
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.dim = dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x


class FullyConnectedFeatureNetwork(FeatureNetwork):
    def __init__(self, sizes: list[int], activation: Type[nn.Module] = nn.GELU, dropout: float = 0.0,
                 batch_norm: bool = False) -> None:
        super().__init__()
        self.input_size = sizes[0]
        self.output_size = sizes[-1]
        self.output_size_lin = sizes[-1]
        self.nn = nn.Sequential()
        if len(sizes) < 2:
            self.nn.append(nn.Identity())
            return
        for a, b in zip(sizes[:-2], sizes[1:-1]):
            self.nn.append(HIPLinear(a, b))
            if batch_norm:
                self.nn.append(nn.BatchNorm1d(b))
            self.nn.append(activation())
            if dropout > 0.0:
                self.nn.append(nn.Dropout(dropout))
        self.nn.append(HIPLinear(sizes[-2], sizes[-1]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.nn(x.view(x.size(0), -1))


class LSTMFeatureNetwork(FeatureNetwork):
    def __init__(self, input_size: int, hidden_size: int, output_size: int, num_layers: int, dropout: float = 0.0,
                 bidirectional: bool = False, pooling: str = "mean", pool_dim: int = 0) -> None:
        super().__init__()
        if pooling not in ("mean", "max"):
            raise ValueError(f'Pooling method {pooling} not supported. Use either "mean" or "max".')
        self.input_size = input_size
        self.output_size = output_size
        self.lstm = nn.LSTM(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers, dropout=dropout,
                            bidirectional=bidirectional, batch_first=True)
        self.linear = nn.Linear(hidden_size * (2 if bidirectional else 1), output_size)
        self.pooling = pooling
        self.pool_dim = pool_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x, _ = self.lstm(x)
        x = self.linear(x)
        if self.pooling == "mean":
            return x.mean(dim=self.pool_dim)
        return x.max(dim=self.pool_dim).values


class FeatureNetworkStack(FeatureNetwork):
    def __init__(self, feature_networks: list[nn.Module | None] | None = None) -> None:
        super().__init__()
        if feature_networks is None or all(fn is None for fn in feature_networks):
            raise ValueError("Feature network stack must contain at least one feature network.")
        self.feature_networks = nn.Sequential(*[fn for fn in feature_networks if fn is not None])
        self.n_distinct_conditions = sum(isinstance(fn, ConcatenateCondition) for fn in self.feature_networks)
        self.input_size = getattr(self.feature_networks[0], "input_size", None)
        self.output_size = getattr(self.feature_networks[-1], "output_size", None)

    def forward(self, *conditions: torch.Tensor) -> torch.Tensor:
        if len(conditions) != self.n_distinct_conditions:
            raise ValueError(f"Expected {self.n_distinct_conditions} conditions, but got {len(conditions)}.")
        feats = None
        used = 0
        for fn in self.feature_networks:
            if isinstance(fn, ConcatenateCondition):
                c = conditions[used]
                feats = fn(c) if feats is None else fn(torch.cat([feats, c], dim=fn.dim))
                used += 1
            else:
                feats = fn(feats)
        return feats


FEATURE_NETWORKS: dict[str, Any] = {
    "FullyConnected": FullyConnectedFeatureNetwork,
    "LSTM": LSTMFeatureNetwork,
    "ConcatenateCondition": ConcatenateCondition,
}

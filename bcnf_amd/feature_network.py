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

import os
import weakref
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


class _LinearGeluFn(torch.autograd.Function):
    """a = dropout(GELU(x W^T + b)) in ONE launch (bcnf_linear_gelu_forward), the backward from the saved
    g = mask GELU'(pre) in the dX / dW GEMMs' operand loads (bcnf_linear_gelu_backward): no ATen GELU, dropout,
    GELU-backward or masked-scale launches."""

    @staticmethod
    def forward(ctx, x, weight, bias, p, rng, salt, need_g):
        from bcnf_amd import _native as N
        rows, k = x.shape
        n = weight.shape[0]
        a = torch.empty((rows, n), dtype=torch.float32, device=x.device)
        g = torch.empty_like(a) if need_g else None
        N.check(N.lib().bcnf_linear_gelu_forward(N.ptr(x), N.ptr(weight), N.ptr(bias), rows, k, n, float(p),
                                                 N.ptr(rng), int(salt), N.ptr(a), N.ptr(g),
                                                 N.stream_handle(x.device)), "bcnf_linear_gelu_forward")
        ctx.save_for_backward(x, weight, g)
        ctx.has_bias = bias is not None
        return a

    @staticmethod
    def backward(ctx, da):
        from bcnf_amd import _native as N
        x, weight, g = ctx.saved_tensors
        if g is None:
            raise RuntimeError("bcnf_amd: fused Linear + GELU layer ran without saving its derivative")
        da = da.contiguous()
        rows, k = x.shape
        n = weight.shape[0]
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dx = torch.empty_like(x) if need_x else None
        dw = torch.empty_like(weight) if (need_w or need_b) else None
        db = torch.empty(n, dtype=torch.float32, device=x.device) if (need_b and ctx.has_bias) else None
        work = None
        if dw is not None:
            wb = int(N.lib().bcnf_linear_work_bytes(rows, k, n))
            work = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=x.device)
        N.check(N.lib().bcnf_linear_gelu_backward(N.ptr(x), N.ptr(weight), N.ptr(da), N.ptr(g), rows, k, n, N.ptr(dx),
                                                  N.ptr(dw), N.ptr(db), N.ptr(work), N.stream_handle(x.device)),
                "bcnf_linear_gelu_backward")
        return dx, (dw if need_w else None), db, None, None, None, None


class HIPLinear(nn.Linear):
    """nn.Linear (same parameters / state_dict keys) whose fp32 GPU forward and backward run on the
    library's MFMA GEMM kernels; other devices / dtypes use torch's own linear."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and self.weight.dtype == torch.float32:
            return _LinearFn.apply(x.contiguous(), self.weight, self.bias)
        return super().forward(x)


# feature network -> weakref to the CondRealNVP_v2 whose coupling Philox state its fused dropout shares
_RNG_OWNERS: "weakref.WeakKeyDictionary[nn.Module, weakref.ref]" = weakref.WeakKeyDictionary()


def bind_rng_owner(fn: nn.Module, owner: nn.Module) -> None:
    _RNG_OWNERS[fn] = weakref.ref(owner)


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
        return self.run(x.view(x.size(0), -1))

    # Philox stream of the fused dropout: the owning CondRealNVP_v2's coupling (seed, offset) state when one is bound
    # (bind_rng_owner; a registry outside the module, so deepcopy / pickle of this module never carry a reference to
    # another model -- CondRealNVP_v2 re-binds its copies), so one device offset serves the feature and the coupling
    # dropout and `model.fused.set_seed` / TrainStep's snapshot cover both; else this module's own state.
    # Advancing: the owner's coupling launch bumps the shared offset once per training step when the coupling itself
    # drops out (and a feature draw that no coupling launch followed -- this network run on its own -- is advanced
    # at the next draw, FusedStack.feature_rng_state); otherwise (coupling dropout 0, the owner in eval mode or
    # elsewhere, no owner) run() bumps it after the network's last fused dropout layer -- a device-side add,
    # replay-safe in HIP graphs -- so every training step draws fresh feature masks.
    _own_rng = None

    def rng_state(self, device) -> torch.Tensor:
        return self._rng(device, draw=False)[0]

    def _rng(self, device, draw: bool = True) -> tuple[torch.Tensor, bool]:
        """(device (seed, offset) state, whether the owner's coupling launch advances it this step); draw: the
        caller draws from it now (marks the draw on the owner's stack, see FusedStack.feature_rng_state)."""
        ref = _RNG_OWNERS.get(self)
        owner = ref() if ref is not None else None
        fused = owner.__dict__.get("_fused") if owner is not None else None
        if fused is not None and hasattr(fused, "rng_state") and getattr(fused, "flat", None) is not None \
                and fused.flat.device == device:
            cfg = getattr(fused, "cfg", None)
            if not draw:
                return fused._rng_tensor(), False
            if owner.training and cfg is not None and cfg.dropout > 0.0:
                return fused.feature_rng_state(), True
            return fused._rng_tensor(), False
        if self._own_rng is None or self._own_rng.device != device:
            seed = (torch.cuda.initial_seed() * 0x9E3779B97F4A7C15 + 0xFEA7) & ((1 << 62) - 1)
            self._own_rng = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        return self._own_rng, False

    def run(self, x: torch.Tensor, upto: int | None = None) -> torch.Tensor:
        """Modules [0, upto) of the MLP on the flattened input. Each Linear -> GELU(exact) [-> Dropout] group of fp32
        CUDA tensors runs as ONE fused launch (bcnf_linear_gelu_forward, salt = its module index); the rest as the
        modules themselves (BatchNorm, other activations, CPU)."""
        mods = list(self.nn)[:upto]
        i = 0
        bump = None                       # the state to advance after the last fused dropout layer, if run() must
        rng = None                        # one state lookup per call (the owner's feature_rng_state marks one draw)
        while i < len(mods):
            m = mods[i]
            act = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, nn.Linear) and isinstance(act, nn.GELU) and act.approximate == "none" \
                    and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and m.weight.dtype == torch.float32:
                drop = mods[i + 2] if i + 2 < len(mods) and isinstance(mods[i + 2], nn.Dropout) else None
                p = drop.p if (drop is not None and drop.training) else 0.0
                if p > 0.0 and rng is None:
                    rng, owner_bumps = self._rng(x.device)
                    bump = None if owner_bumps else rng
                need_g = torch.is_grad_enabled() and (x.requires_grad or m.weight.requires_grad or
                                                      (m.bias is not None and m.bias.requires_grad))
                x = _LinearGeluFn.apply(x.contiguous(), m.weight, m.bias, p, rng if p > 0.0 else None, i, need_g)
                i += 3 if drop is not None else 2
                continue
            x = m(x)
            i += 1
        if bump is not None:
            bump[1:2].add_(1)
        return x


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

    # The LSTM itself stays on PyTorch-ROCm (north star): MIOpen's fused RNN kernels by default; False runs torch's
    # native per-step GEMM + pointwise kernels instead (BCNF_LSTM_MIOPEN=0; tools/gpu_r04.sh lstmab measures both).
    use_miopen = os.environ.get("BCNF_LSTM_MIOPEN", "1") != "0"

    def lstm_out(self, x: torch.Tensor) -> torch.Tensor:
        """The LSTM's output sequence (B, T, hidden * directions)."""
        if self.use_miopen or not x.is_cuda:
            return self.lstm(x)[0]
        with torch.backends.cudnn.flags(enabled=False):
            return self.lstm(x)[0]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.linear(self.lstm_out(x))
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

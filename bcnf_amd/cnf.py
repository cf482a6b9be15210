"""CondRealNVP_v2 and its layers — the reference API (src/bcnf/models/cnf.py) on MI355X HIP kernels.

The module tree, constructor arguments, RNG consumption order at construction, attribute names and
state_dict keys are those of the reference, so checkpoints load in both directions and
`bcnf.train.Trainer` drives this model unchanged. What differs is where the arithmetic runs:

* `CondRealNVP_v2.forward / inverse / sample / log_prob` run the whole coupling stack (ActNorm,
  nested MLP, affine coupling, log|det J|, orthonormal mix) in ONE fused HIP launch
  (bcnf_amd/csrc/bcnf_stack.hip, via the C-ABI in include/bcnf_amd.h); the backward is one more launch
  plus a deterministic gradient reduction.
* A standalone `ConditionalAffineCouplingLayer` runs on the same kernels (a one-block stack).
* The feature networks stay PyTorch-ROCm (north star); their output h is the stack's input.

There is no CPU path for the coupling stack: CPU tensors raise.
"""
from __future__ import annotations

import math
from abc import abstractmethod
from typing import Any

import numpy as np

import torch
import torch.nn as nn

from bcnf_amd.factories import FeatureNetworkFactory, LayerFactory
from bcnf_amd.feature_network import (ConcatenateCondition, FeatureNetwork, FeatureNetworkStack,
                                      FullyConnectedFeatureNetwork, HIPLinear, LSTMFeatureNetwork, bind_rng_owner)
from bcnf_amd.fft_stack import FFTWideStack
from bcnf_amd.fused import FusedStack, StackConfig, stack_forward, stack_inverse, stack_nll, stack_nll_fold
from bcnf_amd.layers import AnyGLU, LinearFFTEnriched
from bcnf_amd.wide import WideStack, make_stack, stack_nll_wide_fold
from bcnf_amd.utils import ParameterIndexMapping, inn_nll_loss, log_prob_from_latent


class InvertibleLayer(nn.Module):
    log_det_J: Any
    n_conditions: int

    @property
    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    @abstractmethod
    def forward(self, y: torch.Tensor, log_det_J: bool = False) -> torch.Tensor:  # pragma: no cover
        pass

    @abstractmethod
    def inverse(self, z: torch.Tensor) -> torch.Tensor:  # pragma: no cover
        pass


class ConditionalInvertibleLayer(nn.Module):
    log_det_J: Any
    n_conditions: int
    device: str

    @property
    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    @abstractmethod
    def forward(self, y: torch.Tensor, x: torch.Tensor, log_det_J: bool = False) -> torch.Tensor:  # pragma: no cover
        pass

    @abstractmethod
    def inverse(self, z: torch.Tensor, x: torch.Tensor) -> torch.Tensor:  # pragma: no cover
        pass


class ConditionalNestedNeuralNetwork(nn.Module):
    """Parameter container with the reference's Sequential layout (cnf.py:49-95): for every hidden size
    Linear, activation, [Dropout if p > 0]; then the final Linear. Its arithmetic runs inside the
    fused HIP coupling kernel (GELU + Linear only)."""

    def __init__(self, sizes: list[int], n_conditions: int, n_output_parameters: int, layer: str = "Linear",
                 layer_kwargs: dict | None = None, activation: str = "GELU", activation_kwargs: dict | None = None,
                 dropout: float = 0.0, device: str = "cpu") -> None:
        super().__init__()
        self.n_conditions = n_conditions
        self.n_output_parameters = n_output_parameters
        self.device = device
        self.dropout = dropout
        self.layer_name = layer
        self.activation_name = activation
        self.nn = nn.Sequential()
        if len(sizes) < 2:
            self.nn.append(nn.Identity())
            return
        sizes = list(sizes)
        sizes[0] += n_conditions
        sizes[-1] *= n_output_parameters
        for a, b in zip(sizes[:-2], sizes[1:-1]):
            self.nn.append(LayerFactory.get_layer(layer, a, b, **(layer_kwargs or {})))
            self.nn.append(LayerFactory.get_layer(activation, **(activation_kwargs or {})))
            if dropout > 0.0:
                self.nn.append(nn.Dropout(dropout))
        self.nn.append(LayerFactory.get_layer(layer, sizes[-2], sizes[-1], **(layer_kwargs or {})))

    @property
    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def linears(self) -> list[nn.Linear]:
        """The Linear of every layer: nn.Linear itself, or a LinearFFTEnriched's inner `linear`."""
        return [m.linear if isinstance(m, LinearFFTEnriched) else m for m in self.nn
                if isinstance(m, (nn.Linear, LinearFFTEnriched))]

    def canonical_params(self) -> list[nn.Parameter]:
        out = []
        for lin in self.linears():
            out += [lin.weight, lin.bias]
        return out

    def fft_widths(self) -> list[int | None]:
        """Per canonical parameter: the input width n of a LinearFFTEnriched weight, else None."""
        out = []
        for m in self.nn:
            if isinstance(m, LinearFFTEnriched):
                out += [m.input_size, None]
            elif isinstance(m, nn.Linear):
                out += [None, None]
        return out

    def forward(self, y: torch.Tensor, h: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """cnf.py:98-107, layer by layer (the "layerwise" path of AnyGLU stacks; the fused families never call it):
        t, tanh(s) from nn(cat(y, h))."""
        if self.n_conditions > 0:
            y = torch.cat([y, h], dim=1)
        t, s = self.nn(y).chunk(2, dim=1)
        return t, torch.tanh(s)


def _coupling_path(layer: str, activation: str, layer_kwargs, activation_kwargs) -> str:
    """Which implementation runs a coupling stack: "fused" (Linear + GELU: the small or wide HIP kernel family),
    "fft" (LinearFFTEnriched + GELU: the wide family on the folded weights, bcnf_amd/fft_stack.py) or "layerwise"
    (AnyGLU: the reference's layer sequence on the GPU, its Linear layers on the library's MFMA GEMMs).
    AnyGLU runs whatever activation module LayerFactory builds (e.g. Identity in
    trajectory_SFrExp_LSTM_SiGLU_2_large.yaml); only the fused and fft paths are tied to GELU."""
    if layer == "AnyGLU":
        return "layerwise"
    if activation != "GELU" or activation_kwargs:
        raise NotImplementedError(f"bcnf_amd's coupling kernels implement activation='GELU' (exact erf); got "
                                  f"activation={activation!r}")
    if layer == "Linear" and not layer_kwargs:
        return "fused"
    if layer == "LinearFFTEnriched" and not layer_kwargs:
        return "fft"
    raise NotImplementedError(f"bcnf_amd: no coupling path implements layer={layer!r} with {layer_kwargs!r}")


def _check_fused_family(layer: str, activation: str, layer_kwargs, activation_kwargs, two_way: bool):
    if _coupling_path(layer, activation, layer_kwargs, activation_kwargs) != "fused":
        raise NotImplementedError(
            f"bcnf_amd: a standalone coupling layer runs on the fused Linear + GELU kernels; layer={layer!r} couplings "
            f"run inside CondRealNVP_v2")


class ConditionalAffineCouplingLayer(ConditionalInvertibleLayer):
    """Affine coupling (cnf.py:110-213). Forward z_b = exp(tanh s') y_b + t, z_a = y_a; inverse
    y_b = (z_b - t) exp(-tanh s'). Standalone calls run the fused HIP kernel as a one-block stack."""

    def __init__(self, input_size: int, nested_sizes: list[int], n_conditions: int, layer: str = "Linear",
                 layer_kwargs: dict | None = None, activation: str = "GELU", activation_kwargs: dict | None = None,
                 dropout: float = 0.0, device: str = "cpu", two_way: bool = False) -> None:
        super().__init__()
        self.n_conditions = n_conditions
        self.log_det_J = torch.zeros(1).to(device)
        self.device = device
        self.two_way = two_way
        self.input_size = input_size
        self.nested_sizes = list(nested_sizes)
        self.dropout = dropout
        self._fam = (layer, activation, layer_kwargs, activation_kwargs)
        da, db = int(np.ceil(input_size / 2)), int(np.floor(input_size / 2))
        self.nn_a = ConditionalNestedNeuralNetwork([da] + list(nested_sizes) + [db], n_conditions, 2, layer,
                                                   layer_kwargs, activation, activation_kwargs, dropout, device)
        if two_way:
            self.nn_b = ConditionalNestedNeuralNetwork([db] + list(nested_sizes) + [da], n_conditions, 2, layer,
                                                       layer_kwargs, activation, activation_kwargs, dropout, device)

    def to(self, *args, **kwargs):  # keep the reference's `.device` bookkeeping (cnf.py:146-155)
        super().to(*args, **kwargs)
        dev = _device_of(args, kwargs)
        if dev is not None:
            self.device = dev
            self.log_det_J = self.log_det_J.to(dev)
        return self

    def canonical_params(self) -> list[nn.Parameter]:
        return self.nn_a.canonical_params()

    def _standalone(self) -> tuple[FusedStack, torch.Tensor]:
        _check_fused_family(*self._fam, self.two_way)
        cfg = StackConfig(self.input_size, tuple(self.nested_sizes), 1, self.n_conditions, self.dropout, False,
                          self.two_way)
        key = (cfg, )
        st = getattr(self, "_solo", None)
        if st is None or st[0] != key:
            st = (key, make_stack(cfg, [], [], bind=False))
            object.__setattr__(self, "_solo", st)
        if not st[1].supported:
            raise NotImplementedError(f"bcnf_amd: no HIP kernel family implements this coupling shape ({cfg})")
        params = self.canonical_params() + (self.nn_b.canonical_params() if self.two_way else [])
        flat = torch.cat([p.reshape(-1) for p in params])
        return st[1], flat

    def forward(self, y: torch.Tensor, x: torch.Tensor, log_det_J: bool = False) -> torch.Tensor:
        if y.dim() == 1:
            y = y.unsqueeze(0)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        stack, flat = self._standalone()
        z, ldj = stack_forward(stack, y, x, self.training, flat=flat)
        if log_det_J:
            self.log_det_J = ldj
        return z

    def inverse(self, z: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        stack, flat = self._standalone()
        return stack_inverse(stack, z, y, training=self.training, flat=flat.detach())

    # the layerwise path (AnyGLU couplings): cnf.py:165-213 as written, on the GPU
    def layerwise_forward(self, y: torch.Tensor, x: torch.Tensor):
        y_a, y_b = y.chunk(2, dim=-1)
        t_a, log_s_a = self.nn_a(y_a, x)
        z_b = torch.exp(log_s_a) * y_b + t_a
        ldj = log_s_a.sum(dim=-1)
        if self.two_way:
            t_b, log_s_b = self.nn_b(z_b, x)
            z_a = torch.exp(log_s_b) * y_a + t_b
            ldj = ldj + log_s_b.sum(dim=-1)
        else:
            z_a = y_a
        return torch.cat([z_a, z_b], dim=-1), ldj

    def layerwise_inverse(self, z: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        z_a, z_b = z.chunk(2, dim=-1)
        t_a, log_s_a = self.nn_a(z_a, y)
        y_b = (z_b - t_a) * torch.exp(-log_s_a)
        if self.two_way:
            t_b, log_s_b = self.nn_b(y_b, y)        # the reference's two_way inverse, as written (cnf.py:206-208)
            y_a = (z_a - t_b) * torch.exp(-log_s_b)
        else:
            y_a = z_a
        return torch.cat([y_a, y_b], dim=-1)


class OrthonormalTransformation(ConditionalInvertibleLayer):
    """Frozen random orthonormal mix y @ Q (cnf.py:312-339). Q = qr(randn(D, D))[0] from the global CPU
    generator, re-seeded with `random_state` when given (bit-identical to the reference)."""

    def __init__(self, input_size: int, random_state: int | None = None) -> None:
        super().__init__()
        self.log_det_J: float = 0
        self.device: str = "cpu"
        if random_state is not None:
            torch.manual_seed(random_state)
        self.orthonormal_matrix = nn.Parameter(torch.linalg.qr(torch.randn(input_size, input_size))[0],
                                               requires_grad=False)

    def forward(self, y: torch.Tensor, x: torch.Tensor, log_det_J: bool = False) -> torch.Tensor:
        return y @ self.orthonormal_matrix

    def inverse(self, z: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        return z @ self.orthonormal_matrix.T


class ActNorm(InvertibleLayer):
    """Per-dimension affine scale*x + bias, log|det J| = sum log|scale| (cnf.py:342-354)."""

    def __init__(self, size: int) -> None:
        super().__init__()
        self.scale = nn.Parameter(torch.ones(size))
        self.bias = nn.Parameter(torch.zeros(size))

    def forward(self, x: torch.Tensor, log_det_J: bool = False) -> torch.Tensor:
        self.log_det_J = torch.sum(torch.log(torch.abs(self.scale)), dim=-1)
        return self.scale * x + self.bias

    def inverse(self, z: torch.Tensor) -> torch.Tensor:
        return (z - self.bias) / self.scale


def _device_of(args, kwargs):
    dev = kwargs.get("device")
    for a in args:
        if isinstance(a, (str, torch.device)):
            dev = a
    if dev is None:
        return None
    return str(dev)


class CondRealNVP_v2(ConditionalInvertibleLayer):
    """Conditional RealNVP (cnf.py:357-588) with the coupling stack on fused MI355X HIP kernels."""

    def __init__(self, size: int, nested_sizes: list[int], n_blocks: int, n_conditions: int,
                 feature_networks: list[FeatureNetwork | nn.Module | None] | None = None, dropout: float = 0.0,
                 act_norm: bool = False, two_way: bool = False, layer: str = "Linear",
                 layer_kwargs: dict[str, Any] | None = None, activation: str = "GELU",
                 activation_kwargs: dict[str, Any] | None = None, device: str = "cpu",
                 random_state: int | None = None, parameter_index_mapping: ParameterIndexMapping | None = None,
                 hybrid: bool = False) -> None:
        super().__init__()
        if n_conditions > 0:
            self.feature_network_stack = FeatureNetworkStack(feature_networks)
        self.size = size
        self.nested_sizes = list(nested_sizes)
        self.n_blocks = n_blocks
        self.n_conditions = n_conditions
        self.device = device
        self.dropout = dropout
        self.act_norm = act_norm
        self.two_way = two_way
        self.parameter_index_mapping = parameter_index_mapping
        self.hybrid = hybrid
        self.log_det_J: torch.Tensor = torch.zeros(1).to(self.device)
        self._fam = (layer, activation, layer_kwargs, activation_kwargs)

        if self.hybrid:
            self.prediction_head = nn.Linear(self.n_conditions, self.size)

        # Same construction (and CPU-RNG consumption) order as cnf.py:395-423.
        self.layers = nn.ModuleList()
        coupling_kwargs = dict(layer=layer, layer_kwargs=layer_kwargs, activation=activation,
                               activation_kwargs=activation_kwargs, dropout=self.dropout, two_way=two_way,
                               device=self.device)
        for _ in range(self.n_blocks - 1):
            if act_norm:
                self.layers.append(ActNorm(self.size))
            self.layers.append(ConditionalAffineCouplingLayer(self.size, self.nested_sizes, self.n_conditions,
                                                              **coupling_kwargs))
            self.layers.append(OrthonormalTransformation(self.size, random_state=random_state))
        self.layers.append(ConditionalAffineCouplingLayer(self.size, self.nested_sizes, self.n_conditions,
                                                          **coupling_kwargs))
        self._build_fused()
        self._bind_feature_rng()

    def _bind_feature_rng(self):
        """The fused feature dropout draws from this model's coupling device Philox state (bind_rng_owner)."""
        fns = getattr(self, "feature_network_stack", None)
        if self.n_conditions > 0 and fns is not None:
            for fn in fns.feature_networks:
                if isinstance(fn, FullyConnectedFeatureNetwork):
                    bind_rng_owner(fn, self)

    # copy.deepcopy / pickle: the fused stack (ctypes descriptor, flat buffers whose views ARE the parameters, a grad
    # hook bound to this model's stack) is not copied; the copy rebuilds its own over its copied parameters and carries
    # the stack's gradient mode and dropout Philox state (seed, device offset), and its feature networks follow the
    # copy's state
    def __getstate__(self):
        state = self.__dict__.copy()
        fused = state.pop("_fused", None)
        if fused is not None:
            rng = getattr(fused, "_rng_state", None)
            state["_fused_carry"] = (getattr(fused, "grad_mode", None), getattr(fused, "seed", None),
                                     rng.detach().clone() if rng is not None else None)
        return state

    def __setstate__(self, state):
        carry = state.pop("_fused_carry", None)
        super().__setstate__(state)
        if carry is not None:
            self._build_fused()
            fused = self._fused
            grad_mode, seed, rng = carry
            if grad_mode is not None and hasattr(fused, "grad_mode"):
                fused.grad_mode = grad_mode
            if hasattr(fused, "seed"):
                fused.seed = seed
            if rng is not None and getattr(fused, "flat", None) is not None:
                fused._rng_state = rng.to(fused.flat.device)
        self._bind_feature_rng()

    # ------------------------------------------------------------------ fused stack plumbing
    def _canonical(self):
        trainable, frozen = [], []
        for layer in self.layers:
            if isinstance(layer, ActNorm):
                trainable += [layer.scale, layer.bias]
            elif isinstance(layer, ConditionalAffineCouplingLayer):
                trainable += layer.canonical_params()
                if layer.two_way:
                    trainable += layer.nn_b.canonical_params()
            elif isinstance(layer, OrthonormalTransformation):
                frozen.append(layer.orthonormal_matrix)
        return trainable, frozen

    def _build_fused(self):
        cfg = StackConfig(self.size, tuple(self.nested_sizes), self.n_blocks, self.n_conditions, self.dropout,
                          self.act_norm, self.two_way)
        trainable, frozen = self._canonical()
        self._path = _coupling_path(*self._fam)
        if self._path == "layerwise":
            object.__setattr__(self, "_fused", _LayerwiseStack(self))
        elif self._path == "fft":
            fft_n = []
            for layer in self.layers:
                if isinstance(layer, ActNorm):
                    fft_n += [None, None]
                elif isinstance(layer, ConditionalAffineCouplingLayer):
                    fft_n += layer.nn_a.fft_widths() + (layer.nn_b.fft_widths() if layer.two_way else [])
            object.__setattr__(self, "_fused", FFTWideStack(cfg, trainable, frozen, fft_n))
        else:
            object.__setattr__(self, "_fused", make_stack(cfg, trainable, frozen))

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        fused = self.__dict__.get("_fused")
        if fused is not None:
            fused.flatten()
        return out

    @property
    def fused(self) -> FusedStack:
        return self._fused

    def flat_parameters(self) -> list[nn.Parameter]:
        """Optimizer-friendly parameter list: ONE flat leaf for the whole coupling stack plus the feature
        network (and prediction head) parameters. Switches the stack to flat-gradient mode."""
        if self._path == "layerwise":
            raise NotImplementedError("bcnf_amd: flat_parameters() needs a fused coupling stack (Linear or "
                                      "LinearFFTEnriched); AnyGLU stacks keep per-layer parameters -- use "
                                      "model.parameters()")
        self._fused.grad_mode = "flat"
        out = [self._fused.flat_param]
        if self.n_conditions > 0:
            out += [p for p in self.feature_network_stack.parameters() if p.requires_grad]
        if self.hybrid:
            out += list(self.prediction_head.parameters())
        return out

    def _check_supported(self):
        if self.n_conditions <= 0:
            # cnf.py:479-485: with n_conditions == 0 no layer matches and the reference raises
            raise ValueError("Layer must be an instance of ConditionalInvertibleLayer or InvertibleLayer, but got "
                             f"{type(self.layers[0])}")
        if self._path == "layerwise":
            return
        if not self._fused.supported:
            raise NotImplementedError(
                "bcnf_amd: this stack shape fits neither HIP kernel family: the register-resident small family "
                "(hidden sizes <= 16, size <= 32, n_conditions <= 256, one-way) nor the wide-MLP MFMA family (equal "
                "nested sizes, size <= 32; one-way or two_way)")

    # ------------------------------------------------------------------ reference API
    def verify(self) -> None:
        current = None
        for fn in self.feature_network_stack.feature_networks:
            if isinstance(fn, FeatureNetwork):
                if current is not None:
                    assert current == fn.input_size, (
                        "The output dimension of the feature network must match the input dimension of the time "
                        f"series network. Have {current} but need {fn.input_size} for next layer.")
                current = fn.output_size
        if current is not None:
            assert current == self.n_conditions, (
                "The output dimension of the time series network must match the number of conditions. "
                f"Have {current} but need {self.n_conditions}.")

    @classmethod
    def from_config(cls, config: dict[str, Any]) -> "CondRealNVP_v2":
        feature_networks = [FeatureNetworkFactory.get_feature_network(fc["type"], fc.get("kwargs", {}))
                            for fc in config["feature_networks"]]
        cnf = cls(feature_networks=feature_networks,
                  parameter_index_mapping=ParameterIndexMapping(list(config["global"]["parameter_selection"])),
                  **config["model"]["kwargs"])
        cnf.verify()
        return cnf

    def to(self, *args, **kwargs) -> "CondRealNVP_v2":
        super().to(*args, **kwargs)
        dev = _device_of(args, kwargs)
        if dev is not None:
            self.device = dev
            self.log_det_J = self.log_det_J.to(dev)
            for layer in self.layers:
                if hasattr(layer, "device"):
                    layer.device = dev
        return self

    @property
    def n_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def _features(self, conditions, deterministic_features=False):
        if deterministic_features:
            self.feature_network_stack.eval()
            return self.feature_network_stack(*conditions).detach()
        return self.feature_network_stack(*conditions)

    def forward(self, y: torch.Tensor, *conditions: torch.Tensor, log_det_J: bool = False,
                return_features: bool = False, deterministic_features: bool = False):
        self._check_supported()
        condition = self._features(conditions, deterministic_features)
        if y.dim() == 1:
            y = y.unsqueeze(0)
        if self._path == "layerwise":
            z, ldj = self._fused.forward(y, condition)
        else:
            z, ldj = stack_forward(self._fused, y, condition, self.training)
        if log_det_J:
            self.log_det_J = ldj
        if return_features:
            return z, condition
        return z

    def nll_loss(self, y: torch.Tensor, *conditions: torch.Tensor, defer_reduction: bool = False,
                 gather=None) -> torch.Tensor:
        """The Trainer's training loss in one fused pass (trainer.py:260-266 with hybrid_weight = 0):
        returns vals = [loss, nll, mse] where loss = nll = inn_nll_loss(z, log_det_J) and mse = 0.
        `vals` is differentiable (backprop loss via vals[0] or with cotangent [1, 0, 0]); the feature
        network runs through autograd as usual, the coupling stack and the loss through the fused
        kernels with no dz / dldj tensors in between. defer_reduction=True (a backward certainly follows)
        moves the loss reduction into the backward launch; vals is then valid only after backward.
        `gather` (TrainStep, folded path only): the batch gather that fills y and the condition, run inside the
        pack launch."""
        self._check_supported()
        if y.dim() == 1:
            y = y.unsqueeze(0)
        if self._path == "layerwise":
            if gather is not None:
                raise ValueError("bcnf_amd: a deferred batch gather needs the folded feature path")
            z, ldj = self._fused.forward(y, self._features(conditions))
            nll = inn_nll_loss(z, ldj)
            return torch.stack([nll, nll, torch.zeros_like(nll)])
        fold = self._foldable_linear(y, conditions)
        if fold is not None:
            x, lin = fold
            return stack_nll_fold(self._fused, y, x, lin.weight, lin.bias, self.training, defer=defer_reduction,
                                  gather=gather)
        wfold = self._wide_fold(y, conditions)
        if wfold is not None and gather is None:
            x, lin = wfold
            return stack_nll_wide_fold(self._fused, y, x, lin.weight, lin.bias, self.training, defer=defer_reduction)
        if gather is not None:
            raise ValueError("bcnf_amd: a deferred batch gather needs the folded feature path")
        condition = self._features(conditions)
        return stack_nll(self._fused, y, condition, self.training, defer=defer_reduction)

    # The training fast path for a feature stack that is ONE nn.Linear (ConcatenateCondition ->
    # FullyConnected(sizes=[X, C]), trajectory_FC_small): h = x Wf^T + bf only enters the stack through the
    # condition projection, so the Linear is folded into it (include/bcnf_amd.h, bcnf_pack_params_fold) and the
    # feature GEMM, dL/dh and the feature dW split-K leave the step. Same sums, reassociated.
    fold_features = True

    def _fold_linear(self):
        """The feature stack's single nn.Linear when the fold applies to this model's structure, else None."""
        if not self.fold_features or type(self._fused) is not FusedStack:
            return None
        fns = list(self.feature_network_stack.feature_networks)
        if len(fns) != 2 or not isinstance(fns[0], ConcatenateCondition) \
                or not isinstance(fns[1], FullyConnectedFeatureNetwork):
            return None
        mods = list(fns[1].nn)
        if len(mods) != 1 or not isinstance(mods[0], nn.Linear):
            return None
        lin = mods[0]
        if lin.weight.dtype != torch.float32 or not lin.weight.is_cuda:
            return None
        if not self._fused.fold_supported(lin.in_features):
            return None
        return lin

    def _foldable_linear(self, y, conditions):
        if len(conditions) != 1:
            return None
        lin = self._fold_linear()
        if lin is None:
            return None
        c = conditions[0]
        if not c.is_cuda or c.dtype != torch.float32 or c.requires_grad or y.requires_grad or c.dim() < 1:
            return None
        x = c.reshape(c.shape[0], -1)       # a view for TrainStep's padded rows (stride(0) = padded width)
        if x.shape[1] != lin.in_features:
            return None
        return x, lin

    # The wide family's training path: the feature network's LAST Linear (FC_large: 310 -> 1360; LSTM_large with
    # pool_dim=1 and mean pooling: 280 -> 1360, mean over time commutes with it) folds into the condition projection
    # (bcnf_amd/wide.py, bcnf_wide_fold_*): the layers before it run as usual and hand x to the stack.
    def _wide_fold(self, y, conditions):
        if not self.fold_features or type(self._fused) is not WideStack or len(conditions) != 1 or y.requires_grad:
            return None
        c = conditions[0]
        if not c.is_cuda or c.dtype != torch.float32:
            return None
        fns = list(self.feature_network_stack.feature_networks)
        if len(fns) != 2 or not isinstance(fns[0], ConcatenateCondition):
            return None
        fn = fns[1]
        if isinstance(fn, FullyConnectedFeatureNetwork):
            mods = list(fn.nn)
            if not mods or type(mods[-1]) not in (nn.Linear, HIPLinear):
                return None
            x = fn.run(c.reshape(c.shape[0], -1), upto=-1)     # the fused Linear + GELU + Dropout layers
            lin = mods[-1]
        elif isinstance(fn, LSTMFeatureNetwork) and fn.pooling == "mean" and fn.pool_dim == 1:
            x = fn.lstm_out(c).mean(dim=1)
            lin = fn.linear
        else:
            return None
        if lin.weight.dtype != torch.float32 or not lin.weight.is_cuda or x.shape[1] != lin.in_features:
            return None
        return x, lin

    def fold_pool_width(self, cond_pool: torch.Tensor):
        """Row width to zero-pad a device-resident condition pool to (TrainStep.set_pool) so the folded path
        reads its batches with float4 loads: the per-sample size rounded up to 4, or None when the fold does not
        apply or the rows are already aligned."""
        lin = self._fold_linear()
        if lin is None or not cond_pool.is_cuda or cond_pool.dim() < 1 or cond_pool.shape[0] == 0:
            return None
        X = cond_pool[0].numel()
        if X != lin.in_features or X % 4 == 0:
            return None
        return (X + 3) // 4 * 4

    def log_prob(self, y: torch.Tensor, *conditions: torch.Tensor) -> torch.Tensor:
        """log p(y | conditions) = -0.5 |z|^2 + log|det J| - D/2 log(2 pi). The reference has no such
        method; it equals -inn_nll_loss(z, log_det_J, 'none') - D/2 log 2pi (utils.py:49-53)."""
        z = self.forward(y, *conditions, log_det_J=True)
        return log_prob_from_latent(z, self.log_det_J)

    def inverse(self, z: torch.Tensor, *conditions: torch.Tensor) -> torch.Tensor:
        self._check_supported()
        condition = self.feature_network_stack(*conditions)
        if self._path == "layerwise":
            return self._fused.inverse(z, condition)
        return stack_inverse(self._fused, z, condition, training=self.training)

    def _inverse_indexed(self, z, h_unique, cond_index):
        if self._path == "layerwise":
            return self._fused.inverse(z, h_unique[cond_index])
        return stack_inverse(self._fused, z, h_unique, cond_index=cond_index, training=self.training)

    def sample(self, n_samples: int, *conditions: torch.Tensor, sigma: float = 1, outer: bool = False,
               batch_size: int = 100, sample_batch_size: int | None = None, output_device: str = "cpu",
               verbose: bool = False) -> torch.Tensor:
        """cnf.py:510-538: same chunking, same CPU-generator z stream, same output layout."""
        self._check_supported()
        if sample_batch_size is None:
            sample_batch_size = batch_size
        m_sizes = [sample_batch_size] * (n_samples // sample_batch_size) + [n_samples % sample_batch_size]
        rows: list[list[torch.Tensor]] = []
        with torch.no_grad(), self._fused.reuse_pack():
            for b in range(0, len(conditions[0]), batch_size):
                batch_conditions = [c[b: b + batch_size].to(self.device) for c in conditions]
                rows.append([])
                for m in m_sizes:
                    if m == 0:
                        continue
                    rows[-1].append(self._sample(m, *batch_conditions, outer=outer, sigma=sigma).to(output_device))
        return torch.cat([torch.cat(r, dim=0) for r in rows], dim=1)

    def _sample(self, n_samples: int, *conditions: torch.Tensor, sigma: float = 1, outer: bool = False):
        """cnf.py:540-588. Features are computed once per distinct condition; tiled rows index them."""
        if all(c.ndim == 1 for c in conditions):
            z = (sigma * torch.randn(n_samples, self.size)).to(self.device)
            h = self.feature_network_stack(*[c.unsqueeze(0) for c in conditions])
            idx = torch.zeros(n_samples, dtype=torch.int64, device=z.device)
            return self._inverse_indexed(z, h, idx).view(n_samples, self.size)
        if all(c.ndim > 1 for c in conditions):
            if outer:
                if len(set(c.shape[0] for c in conditions)) != 1:
                    raise ValueError("All conditions must have the same number of samples (dim = 0). "
                                     f"Got {[c.shape for c in conditions]}.")
                nc = conditions[0].shape[0]
                z = (sigma * torch.randn(n_samples * nc, self.size)).to(self.device)
                h = self.feature_network_stack(*conditions)
                idx = torch.arange(n_samples * nc, device=z.device, dtype=torch.int64) % nc
                return self._inverse_indexed(z, h, idx).view(n_samples, nc, self.size)
            z = (sigma * torch.randn(n_samples, self.size)).to(self.device)
            h = self.feature_network_stack(*conditions)
            if self._path == "layerwise":
                return self._fused.inverse(z, h).view(n_samples, self.size)
            return stack_inverse(self._fused, z, h, training=self.training).view(n_samples, self.size)
        raise ValueError(f"Conditions have invalid shape: {[c.shape for c in conditions]}")


class _LayerwiseStack:
    """The coupling stack of an AnyGLU model (reference layers.py:9-31, dev configs): the reference's layer sequence
    (cnf.py:467-508) on the GPU, each AnyGLU's two Linear layers on the library's fp32 MFMA GEMMs (HIPLinear), the
    elementwise work in PyTorch-ROCm, gradients by autograd. Not fused: no HIP kernel family implements GLU
    couplings. CPU tensors raise, as on the fused paths."""

    supported = True

    def __init__(self, model: "CondRealNVP_v2"):
        self._model = model

    def _check(self, t: torch.Tensor):
        if not t.is_cuda:
            raise RuntimeError("bcnf_amd: the coupling stack runs on the GPU (MI355X); got a CPU tensor")

    def forward(self, y: torch.Tensor, h: torch.Tensor):
        self._check(y)
        ldj = torch.zeros(y.shape[0], dtype=y.dtype, device=y.device)
        for layer in self._model.layers:
            if isinstance(layer, ActNorm):
                y = layer(y)
                ldj = ldj + torch.sum(torch.log(torch.abs(layer.scale)), dim=-1)
            elif isinstance(layer, ConditionalAffineCouplingLayer):
                y, l = layer.layerwise_forward(y, h)
                ldj = ldj + l
            else:
                y = y @ layer.orthonormal_matrix
        return y, ldj

    def inverse(self, z: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
        self._check(z)
        for layer in reversed(self._model.layers):
            if isinstance(layer, ActNorm):
                z = layer.inverse(z)
            elif isinstance(layer, ConditionalAffineCouplingLayer):
                z = layer.layerwise_inverse(z, h)
            else:
                z = z @ layer.orthonormal_matrix.T
        return z

    def reuse_pack(self):
        import contextlib
        return contextlib.nullcontext(self)

    def flatten(self):
        pass

    def sync_grad_state(self):
        pass

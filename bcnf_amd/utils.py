"""Small host-side utilities mirroring the reference's public helpers on the hot path.

* inn_nll_loss            <- src/bcnf/utils.py:49-53
* ParameterIndexMapping   <- src/bcnf/utils.py:166-196
* load_config             <- src/bcnf/utils.py:13-46 (Dynaconf there; here yaml.safe_load + YAML-1.1
                             number coercion, since Dynaconf is not available offline)
"""
from __future__ import annotations

import math
import os
import re
from typing import Any, Iterator

import numpy as np
import torch
import yaml


def inn_nll_loss(z: torch.Tensor, log_det_J: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """Negative log-likelihood of a standard-normal latent without the Gaussian constant (utils.py:49-53)."""
    per_sample = 0.5 * torch.sum(z ** 2, dim=1) - log_det_J
    if reduction == "mean":
        return torch.mean(per_sample)
    return per_sample


def log_prob_from_latent(z: torch.Tensor, log_det_J: torch.Tensor) -> torch.Tensor:
    """log p(y|x) = -0.5|z|^2 + log|det J| - D/2 log(2 pi)   (SURVEY §8a-10 contract)."""
    return -inn_nll_loss(z, log_det_J, reduction="none") - 0.5 * z.shape[1] * math.log(2.0 * math.pi)


class ParameterIndexMapping:
    """Name <-> column index of the inferred physical parameters (utils.py:166-196)."""

    def __init__(self, parameters: list[str]) -> None:
        self.parameters = list(parameters)
        self.map = {name: i for i, name in enumerate(self.parameters)}

    def __len__(self) -> int:
        return len(self.parameters)

    def vectorize(self, parameter_dict: dict) -> np.ndarray:
        missing = [p for p in self.parameters if p not in parameter_dict]
        if missing:
            raise KeyError(f'Parameter "{missing[0]}" not found in the parameter dictionary. '
                           f'Have available keys: {list(parameter_dict.keys())}')
        return np.array([parameter_dict[p] for p in self.parameters]).T

    def dictify(self, parameter_vector: np.ndarray) -> dict:
        return {name: parameter_vector[i] for i, name in enumerate(self.parameters)}

    def __getitem__(self, key: str) -> int:
        return self.map[key]

    def __iter__(self) -> Iterator[str]:
        return iter(self.parameters)

    def __contains__(self, key: str) -> bool:
        return key in self.map

    def __repr__(self) -> str:
        return str(self.parameters)

    __str__ = __repr__


_FLOAT_RE = re.compile(r"^[-+]?(\d[\d_]*\.?[\d_]*|\.\d[\d_]*)([eE][-+]?\d+)?$")
_INT_RE = re.compile(r"^[-+]?\d[\d_]*$")


def _coerce(v: Any) -> Any:
    """PyYAML safe_load leaves '2e-4' a string (YAML 1.1) while Dynaconf/TOML parse it as a float;
    the reference's Adam then needs a float. Also accept 2024_03_25-style ints."""
    if isinstance(v, dict):
        return {k: _coerce(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_coerce(x) for x in v]
    if isinstance(v, str):
        t = v.strip()
        if _INT_RE.match(t):
            return int(t.replace("_", ""))
        if _FLOAT_RE.match(t) and any(c in t for c in ".eE"):
            return float(t.replace("_", ""))
    return v


def bcnf_root() -> str:
    return os.environ.get("BCNF_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sub_root_path(path: str) -> str:
    return re.sub(r"{{BCNF_ROOT}}", bcnf_root(), path)


def load_config(config_file: str, verify: bool = True) -> dict:
    """Load a run configuration YAML into nested dicts with lower-cased top-level keys (the Trainer
    lower-cases keys too, trainer.py:80)."""
    config_file = sub_root_path(config_file)
    if not os.path.exists(config_file):
        raise FileNotFoundError(f"File '{config_file}' does not exist.")
    with open(config_file) as f:
        cfg = _coerce(yaml.safe_load(f))
    cfg = {str(k).lower(): v for k, v in cfg.items()}
    data = cfg.get("data")
    if isinstance(data, dict):
        for key in ("path", "config_file"):
            if isinstance(data.get(key), str):
                data[key] = sub_root_path(data[key])
    return cfg

"""String -> class factories used by from_config (reference src/bcnf/factories.py:13-73)."""
from __future__ import annotations

from typing import Any, Iterator

import torch
import torch.nn as nn

from bcnf_amd.feature_network import FEATURE_NETWORKS


class SchedulerFactory:
    @staticmethod
    def get_scheduler(scheduler: str, optimizer: torch.optim.Optimizer, scheduler_kwargs: Any):
        if scheduler == "ReduceLROnPlateau":
            return torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, **scheduler_kwargs)
        raise NotImplementedError(f"Scheduler {scheduler} not implemented")


class OptimizerFactory:
    @staticmethod
    def get_optimizer(optimizer: str, parameters: Iterator[nn.Parameter], optimizer_kwargs: Any):
        if optimizer == "Adam":
            return torch.optim.Adam(parameters, **optimizer_kwargs)
        raise NotImplementedError(f"Optimizer {optimizer} not implemented")


class FeatureNetworkFactory:
    @staticmethod
    def get_feature_network(network: str | None, network_kwargs: Any) -> nn.Module:
        if network is None:
            return nn.Identity()
        cls = FEATURE_NETWORKS.get(network)
        if cls is None:
            raise NotImplementedError(f"Feature network {network} not implemented in bcnf_amd")
        return cls(**(network_kwargs or {}))


class LayerFactory:
    """Resolves `layer` / `activation` strings (cnf.py:80-81; factories.py:61-73): torch.nn first, then the
    variant layers of bcnf_amd.layers (AnyGLU, LinearFFTEnriched, ...), as the reference falls back to bcnf.models.
    Which kernel path a coupling stack takes is decided when the model is built (bcnf_amd/cnf.py)."""

    @staticmethod
    def get_layer(layer: str, *args: Any, **kwargs: Any) -> nn.Module:
        if hasattr(nn, layer):
            return getattr(nn, layer)(*args, **kwargs)
        from bcnf_amd.layers import LAYERS
        if layer in LAYERS:
            return LAYERS[layer](*args, **kwargs)
        raise NotImplementedError(f"Layer {layer} not implemented")

"""bcnf_amd — MI355X-native (gfx950 / CDNA4) CondRealNVP_v2 coupling-stack hot path.

Drop-in for psaegert/bcnf's `CondRealNVP_v2` (src/bcnf/models/cnf.py): same constructor, from_config,
forward / inverse / sample API and state_dict layout, with the coupling stack on fused HIP kernels.
"""
from bcnf_amd.cnf import (ActNorm, CondRealNVP_v2, ConditionalAffineCouplingLayer, ConditionalInvertibleLayer,
                          ConditionalNestedNeuralNetwork, InvertibleLayer, OrthonormalTransformation)
from bcnf_amd.feature_network import (ConcatenateCondition, FeatureNetwork, FeatureNetworkStack,
                                      FullyConnectedFeatureNetwork, LSTMFeatureNetwork)
from bcnf_amd.utils import ParameterIndexMapping, inn_nll_loss, load_config, log_prob_from_latent

__all__ = [
    "ActNorm", "CondRealNVP_v2", "ConditionalAffineCouplingLayer", "ConditionalInvertibleLayer",
    "ConditionalNestedNeuralNetwork", "InvertibleLayer", "OrthonormalTransformation", "ConcatenateCondition",
    "FeatureNetwork", "FeatureNetworkStack", "FullyConnectedFeatureNetwork", "LSTMFeatureNetwork",
    "ParameterIndexMapping", "inn_nll_loss", "load_config", "log_prob_from_latent",
]

"""Variant coupling layers on CPU (no kernels run): the rfft matrix of the LinearFFTEnriched fold equals torch.fft,
the layer modules keep the reference's parameter names, and the variant models build with the reference's
state_dict layout (fixtures g12 / g13 from psaegert/bcnf)."""
import copy

import numpy as np
import pytest
import torch

from conftest import load_golden
from test_gpu_variants import CASES


@pytest.mark.parametrize("n", [1, 2, 7, 40, 52, 175])
def test_rfft_matrix_equals_torch_fft(n):
    from bcnf_amd.layers import FFTLayer, rfft_matrix
    x = torch.randn(9, n, dtype=torch.float64)
    assert torch.allclose(x @ rfft_matrix(n, torch.float64).T, FFTLayer()(x), atol=1e-12)


def test_fft_enriched_fold_is_the_layer():
    """W cat(x, F x) + b == (W[:, :n] + W[:, n:] F) x + b: the identity the fused FFT path rests on."""
    from bcnf_amd.layers import LinearFFTEnriched, rfft_matrix
    torch.manual_seed(0)
    lay = LinearFFTEnriched(23, 11).double()
    x = torch.randn(5, 23, dtype=torch.float64)
    W, b = lay.linear.weight, lay.linear.bias
    weff = W[:, :23] + W[:, 23:] @ rfft_matrix(23, torch.float64)
    assert torch.allclose(lay(x), x @ weff.T + b, atol=1e-12)


def test_layer_parameter_names():
    from bcnf_amd.layers import AnyGLU, LinearFFTEnriched
    assert [k for k, _ in AnyGLU(4, 3, activation="Sigmoid").named_parameters()] == [
        "linear_gate.weight", "linear_gate.bias", "linear_value.weight", "linear_value.bias"]
    assert [k for k, _ in LinearFFTEnriched(6, 3).named_parameters()] == ["linear.weight", "linear.bias"]
    assert tuple(LinearFFTEnriched(6, 3).linear.weight.shape) == (3, 6 + 2 * 4)


@pytest.mark.parametrize("name", sorted(CASES))
def test_variant_models_build_with_reference_layout(name):
    from bcnf_amd import CondRealNVP_v2
    cfg, fx, stack = CASES[name]
    d = load_golden(fx)
    m = CondRealNVP_v2.from_config(copy.deepcopy(cfg))
    assert type(m.fused).__name__ == stack
    sd = m.state_dict()
    ref = {k[3:]: d[k] for k in d.keys() if k.startswith("sd/")}
    assert list(sd.keys()) == list(ref.keys())
    for k, v in ref.items():
        assert tuple(sd[k].shape) == v.shape, k
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ref.items()})
    qs = [v for k, v in m.state_dict().items() if k.endswith("orthonormal_matrix")]
    assert all(np.array_equal(q.numpy(), ref[k]) for k, q in zip([k for k in ref if k.endswith("orthonormal_matrix")], qs))


@pytest.mark.parametrize("name", sorted(CASES))
def test_variant_models_refuse_cpu_tensors(name):
    """A model left on the CPU raises a clean RuntimeError on every path -- the FFT path included, whose weight fold
    would otherwise hand host pointers to the HIP GEMM (no kernel runs here)."""
    from bcnf_amd import CondRealNVP_v2
    m = CondRealNVP_v2.from_config(copy.deepcopy(CASES[name][0]))
    with pytest.raises(RuntimeError):
        m.forward(torch.randn(3, 19), torch.randn(3, 12), log_det_J=True)
    with pytest.raises(RuntimeError):
        m.inverse(torch.randn(3, 19), torch.randn(3, 12))


def test_anyglu_identity_activation_builds():
    """trajectory_SFrExp_LSTM_SiGLU_2_large.yaml: layer AnyGLU with activation Identity -- the layerwise path runs
    whatever activation module LayerFactory builds, so the model builds (only the fused / fft paths need GELU)."""
    from bcnf_amd import CondRealNVP_v2
    cfg = copy.deepcopy(CASES["anyglu"][0])
    cfg["model"]["kwargs"]["activation"] = "Identity"
    m = CondRealNVP_v2.from_config(cfg)
    assert type(m.fused).__name__ == "_LayerwiseStack"
    assert any(type(mod).__name__ == "Identity" for mod in m.modules())
    with pytest.raises(NotImplementedError):
        m.flat_parameters()
    cfg["model"]["kwargs"]["layer"] = "Linear"
    cfg["model"]["kwargs"].pop("layer_kwargs")
    with pytest.raises(NotImplementedError):
        CondRealNVP_v2.from_config(cfg)          # the fused Linear kernels implement GELU only

"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/bcnf_amd.h declares, and
its host-side layout queries agree with the PyTorch module tree. No compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "bcnf_amd.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(bcnf_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    from bcnf_amd import _native as N
    lib = N.lib()
    names = header_functions()
    assert len(names) == len(N.EXPORTS) and set(names) == set(N.EXPORTS)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.bcnf_status_string(0) == b"ok"


def test_layout_queries_match_module_tree():
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    cfg = {"global": {"parameter_selection": [str(i) for i in range(19)]},
           "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 7, "n_conditions": 80, "n_blocks": 32,
                                "dropout": 0.383, "act_norm": True}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
    m = CondRealNVP_v2.from_config(cfg)
    ntr, nfr = m.fused.counts()
    assert ntr == m.fused.flat.numel() == 109786
    assert nfr == 31 * 19 * 19 == 11191
    assert m.n_params == 128257
    assert m.fused.supported
    d = m.fused.desc
    ws = N.query_i64(N.lib().bcnf_workspace_bytes, ctypes.byref(d), ctypes.c_int64(4096), ctypes.c_int32(1))
    # activation records (7 masked activations, 7 masked GELU derivatives, tanh(s), y_a, y_b -> 20 floats
    # per lane and block), loss partials, condition projection HP, Linear-1 deltas D1 (+ a dummy row)
    assert ws == 32 * 4096 * 16 * 20 * 4 + 256 * 4 + 2 * 32 * 4096 * 16 * 4 + 16 * 4   # + D1 dummy row
    sb = N.query_i64(N.lib().bcnf_slab_bytes, ctypes.byref(d), ctypes.c_int64(4096))
    # per workgroup: nb blocks of the compact block (3430 - 16*80 condition columns = 2150, padded to 4),
    # plus 32 split-K partials (128 rows each) of the condition columns [nb][16][80]
    assert sb == 256 * 32 * 2152 * 4 + 32 * 32 * 16 * 80 * 4


def test_unsupported_shapes_are_rejected():
    from bcnf_amd import _native as N
    lib = N.lib()
    big = N.make_desc(19, [526] * 5, 26, 1360, 0.407, True)
    assert lib.bcnf_stack_supported(ctypes.byref(big)) == 0
    tw = N.make_desc(19, [16] * 3, 4, 80, 0.0, True, two_way=True)
    assert lib.bcnf_stack_supported(ctypes.byref(tw)) == 0
    bad = N.make_desc(19, [16] * 3, 4, 80, 1.5, True)
    assert lib.bcnf_stack_supported(ctypes.byref(bad)) == 0


def test_cpu_tensors_raise_loudly():
    from bcnf_amd import CondRealNVP_v2
    cfg = {"global": {"parameter_selection": [str(i) for i in range(19)]},
           "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 2, "n_conditions": 80, "n_blocks": 2}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
    m = CondRealNVP_v2.from_config(cfg)
    with pytest.raises(RuntimeError, match="HIP kernels only"):
        m(torch.randn(4, 19), torch.randn(4, 30, 3))


def test_state_dict_roundtrip_keeps_flat_views():
    from bcnf_amd import CondRealNVP_v2
    cfg = {"global": {"parameter_selection": [str(i) for i in range(19)]},
           "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 2, "n_conditions": 80, "n_blocks": 3,
                                "act_norm": True, "dropout": 0.2}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
    torch.manual_seed(1)
    a = CondRealNVP_v2.from_config(cfg)
    torch.manual_seed(2)
    b = CondRealNVP_v2.from_config(cfg)
    b.load_state_dict(a.state_dict())
    flat_a = torch.cat([p.reshape(-1) for p in a.fused.trainable])
    assert torch.equal(b.fused.flat, flat_a)
    assert torch.equal(b.fused.flat, a.fused.flat)
    # the per-layer parameters are views of the flat buffer
    p0 = b.layers[1].nn_a.nn[0].weight
    assert p0.data_ptr() == b.fused.flat.data_ptr() + 2 * 19 * 4
    assert list(a.state_dict().keys())[2:6] == ["layers.0.scale", "layers.0.bias", "layers.1.nn_a.nn.0.weight",
                                                "layers.1.nn_a.nn.0.bias"]

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


def test_boundary_has_no_global_state():
    """stateless entry points. The header declares no process-global setter, no last-error query and no
    debug hook; HIP failures come back in the status code (BCNF_ERR_HIP_BASE + hipError_t); the shipped library
    exports no debug symbols (they exist only in the -DBCNF_PHASE_STAMPS diagnostic build)."""
    from bcnf_amd import _native as N
    names = header_functions()
    for n in names:
        assert not re.search(r"force|set_|debug|last_|_error$", n), n
    src = open(HEADER).read()
    assert "BCNF_ERR_HIP_BASE 1000" in src and N.ERR_HIP_BASE == 1000
    lib = N.lib()
    for n in ("bcnf_last_hip_error", "bcnf_wide_force_tiling", "bcnf_debug_phases", "bcnf_wide_debug_phases"):
        assert not hasattr(lib, n), n
    assert lib.bcnf_status_string(1000 + 98).decode() not in ("ok", "unknown status")   # hipErrorInvalidImage
    for d in ("bcnf_stack.hip", "bcnf_wide.hip", "bcnf_train.hip", "bcnf_device.h"):
        assert "BCNF_EXP" not in open(os.path.join(ROOT, "bcnf_amd", "csrc", d)).read(), d


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
    # activation records ((masked activation, masked GELU derivative) x 7, y_a, y_b, tanh(s) -> 17 floats
    # per lane and block), loss partials, condition projection HP, Linear-1 deltas D1 (+ a dummy row)
    assert ws == 32 * 4096 * 16 * 17 * 4 + 256 * 4 + 2 * 32 * 4096 * 16 * 4 + 16 * 4   # 17-float records, + D1 dummy row
    sb = N.query_i64(N.lib().bcnf_slab_bytes, ctypes.byref(d), ctypes.c_int64(4096))
    # per workgroup: nb blocks of the compact block (3430 - 16*80 condition columns = 2150, padded to 4),
    # plus 32 split-K partials (128 rows each) of the condition columns [nb][16][80]
    assert sb == 256 * 32 * (9 * 256 + 13 * 16) * 4 + 32 * 32 * 16 * 80 * 4   # MFMA tiles + column sums per block


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


def test_wide_family_routing_and_layout_queries():
    """FC_large / LSTM_large shapes route to the wide-MLP family (bcnf_wide.hip); its size queries follow the
    carve-up documented in DESIGN.md (padded activation rows HP = round_up(H + 1, 4))."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd import _native as N
    from bcnf_amd.wide import WideStack
    lib = N.lib()
    big = N.make_desc(19, [526] * 5, 26, 1360, 0.407, True)
    assert lib.bcnf_wide_supported(ctypes.byref(big)) == 1
    for bad in (N.make_desc(19, [526, 500], 2, 1360, 0.0, True),          # unequal nested sizes
                N.make_desc(40, [526] * 2, 2, 1360, 0.0, True)):          # D > 32
        assert lib.bcnf_wide_supported(ctypes.byref(bad)) == 0
    for good in (N.make_desc(19, [526] * 2, 2, 1361, 0.0, True),          # C % 4 != 0 (rows re-laid inside)
                 N.make_desc(19, [336] * 5, 26, 1360, 0.407, True, two_way=True)):   # trajectory_LSTM_2_large
        assert lib.bcnf_wide_supported(ctypes.byref(good)) == 1
    cfg = {"global": {"parameter_selection": [str(i) for i in range(19)]},
           "model": {"kwargs": {"size": 19, "nested_sizes": [526] * 5, "n_conditions": 1360, "n_blocks": 26,
                                "dropout": 0.407, "act_norm": True}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90] + [310] * 7 + [1360],
                                                                      "dropout": 0.111}}]}
    m = CondRealNVP_v2.from_config(cfg)
    assert isinstance(m.fused, WideStack)
    assert m.n_params == 48_865_045                       # SURVEY §8a-1 [measured]
    assert m.fused.flat.numel() == m.fused.counts()[0] == 47_826_390
    HP, nb, NH, B = 528, 26, 5, 2048
    pk = N.query_i64(lib.bcnf_wide_packed_bytes, ctypes.byref(big))
    r4 = lambda n: (n + 3) // 4 * 4  # noqa: E731
    assert pk == 4 * (r4(nb * HP * 1360) + 2 * r4(nb * (NH - 1) * HP * HP) + r4(nb * 10 * HP) + r4(nb * 18 * HP)
                      + r4(25 * 19 * 19) + r4(nb) + nb * HP)
    ws = N.query_i64(lib.bcnf_wide_workspace_bytes, ctypes.byref(big), ctypes.c_int64(B), ctypes.c_int32(1))
    slab = B * HP
    regions = [B * nb * HP, B, nb * NH * slab, nb * NH * slab, nb * (NH - 1) * slab, B * nb * HP, (nb + 1) * B * 20,
               nb * B * 12, nb * B * 12, nb * B * 20, B * 20, nb * B * 40,
               B * 32 * 11]                   # last-Linear partials: 32 floats x ceil(528 / 48) column tiles per row
    assert ws == 4 * sum(r4(n) + 64 for n in regions)
    # the small family keeps FC_small
    small = N.make_desc(19, [16] * 7, 32, 80, 0.383, True)
    assert lib.bcnf_stack_supported(ctypes.byref(small)) == 1


def test_two_way_parameter_layout_matches_module_tree():
    """two_way: each block's nn_b parameters follow its nn_a parameters in the flat buffer (state_dict order), and the
    library's count agrees (dev config trajectory_LSTM_2_large shapes, FC feature net stand-in)."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.wide import WideStack
    cfg = {"global": {"parameter_selection": [str(i) for i in range(19)]},
           "model": {"kwargs": {"size": 19, "nested_sizes": [336] * 5, "n_conditions": 1360, "n_blocks": 3,
                                "dropout": 0.407, "act_norm": True, "two_way": True}},
           "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                                {"type": "FullyConnected", "kwargs": {"sizes": [90, 1360]}}]}
    m = CondRealNVP_v2.from_config(cfg)
    assert isinstance(m.fused, WideStack) and m.fused.supported
    names = [n for n, _ in m.named_parameters() if n.startswith("layers.")]
    assert names[:4] == ["layers.0.scale", "layers.0.bias", "layers.1.nn_a.nn.0.weight", "layers.1.nn_a.nn.0.bias"]
    assert names[2 + 12] == "layers.1.nn_b.nn.0.weight"
    mlp_a = (10 + 1360) * 336 + 336 + 4 * (336 * 336 + 336) + 336 * 18 + 18
    mlp_b = (9 + 1360) * 336 + 336 + 4 * (336 * 336 + 336) + 336 * 20 + 20
    assert m.fused.flat.numel() == m.fused.counts()[0] == 3 * (mlp_a + mlp_b) + 2 * 38
    w_b = m.layers[1].nn_b.nn[0].weight
    assert w_b.data_ptr() == m.fused.flat.data_ptr() + (38 + mlp_a) * 4


def _c_layout(struct, fields):
    """sizeof / offsetof of a struct of include/bcnf_amd.h as the C compiler lays it out (gcc, host)."""
    import subprocess
    import tempfile
    body = "\n".join(f'  printf("%zu\\n", offsetof({struct}, {f}));' for f in fields)
    src = (f'#include <stddef.h>\n#include <stdio.h>\n#include "bcnf_amd.h"\nint main(void) {{\n'
           f'  printf("%zu\\n", sizeof({struct}));\n{body}\n  return 0;\n}}\n')
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        out = [int(v) for v in subprocess.check_output([exe]).split()]
    return out[0], out[1:]


@pytest.mark.parametrize("name", ["BcnfStackDesc", "BcnfGather2", "BcnfFoldAdam"])
def test_ctypes_structs_match_the_c_abi(name):
    """The ctypes mirrors in bcnf_amd/_native.py have the size and field offsets of the header's structs."""
    from bcnf_amd import _native as N
    cls = getattr(N, name)
    fields = [f[0] for f in cls._fields_]
    size, offs = _c_layout(name, fields)
    assert ctypes.sizeof(cls) == size
    assert [getattr(cls, f).offset for f in fields] == offs


def test_fold_adam_spec_host_logic():
    """FusedAdam.fold_adam_spec: pointers of each slot's parameter / moments, the shared step, hyper-parameters;
    None unless the slots are exactly the optimizer's parameters."""
    from bcnf_amd.optim import FusedAdam
    flat, w, b = (torch.nn.Parameter(torch.zeros(n)) for n in (10, 6, 3))
    opt = FusedAdam([flat, w, b], lr=2e-4)
    counter = torch.zeros(1, dtype=torch.int32)
    spec = opt.fold_adam_spec((flat, w, b), counter=counter)
    for t, p in enumerate((flat, w, b)):
        st = opt.state[p]
        assert spec.params[t] == p.data_ptr()
        assert spec.exp_avg[t] == st["exp_avg"].data_ptr() and spec.exp_avg_sq[t] == st["exp_avg_sq"].data_ptr()
        assert st["step"] is opt.state[flat]["step"]
    assert spec.step == opt.state[flat]["step"].data_ptr() and spec.done_counter == counter.data_ptr()
    assert (spec.lr, spec.beta1, spec.beta2, spec.eps) == (2e-4, 0.9, 0.999, 1e-8)
    assert opt.fold_adam_spec((flat, w, None), counter=counter) is None       # b would not be updated
    other = torch.nn.Parameter(torch.zeros(2))
    assert opt.fold_adam_spec((flat, w, other), counter=counter) is None


def test_fold_raw_table_partitions_the_record():
    """bcnf_fold_raw_table (host): every float of a forward record's 16 lanes belongs to exactly one (thread, slot)
    of the pack-free forward's table -- no two helper threads write the same LDS word -- with P-sourced offsets
    inside one block's parameters (sorted: a wave reads consecutive parameters) and Q-sourced ones inside one D x D
    matrix; the backward-record appendix holds one (source, kind) per word; shapes it cannot express are refused."""
    import numpy as np
    from bcnf_amd import _native as N
    L = N.lib()
    for nested, C, X in (([16] * 7, 80, 90), ([16, 8, 12], 13, 21), ([4], 40, 96)):
        d = N.make_desc(19, nested, 32, C, 0.1, True)
        nb = ctypes.c_int64(0)
        assert L.bcnf_fold_raw_table_bytes(ctypes.byref(d), X, ctypes.byref(nb)) == N.OK
        raw = np.zeros(nb.value // 4, dtype=np.uint32)
        assert L.bcnf_fold_raw_table(ctypes.byref(d), X, ctypes.c_void_p(raw.ctypes.data)) == N.OK
        t, pb = raw[:20 * 256].reshape(256, 20)[:, :18].T, raw[20 * 256:]   # [thread][20 slots] -> [slot][thread]
        dst, src = t & 4095, t >> 12
        live = dst != 4095
        words = dst[live]
        assert len(np.unique(words)) == words.size                  # each word once
        assert words.max() + 1 == words.size                        # ... and all of 0 .. 16 RF - 1
        assert words.size % 16 == 0
        n_tr = ctypes.c_int64(0)
        assert L.bcnf_param_count(ctypes.byref(d), ctypes.byref(n_tr), None) == N.OK
        p_src = src[:10][live[:10]]
        assert p_src.max() < n_tr.value // 31                       # within one block's parameters
        assert (np.diff(src[:10].reshape(-1)[live[:10].reshape(-1)].astype(np.int64)) > 0).all()   # sorted, distinct
        assert src[10:12][live[10:12]].max() < 19 * 19
        assert (src[12:][live[12:]] == 0).all()                     # zero words carry no source
        kind = pb & 3
        assert pb.size % 16 == 0 and set(np.unique(kind)) <= {0, 1, 2}
        assert (pb[kind == 0] >> 2).max() < n_tr.value // 31
        assert (pb[kind == 1] >> 2).max() < 19 * 19
    nb = ctypes.c_int64(0)
    no_an = N.make_desc(19, [16] * 7, 32, 80, 0.1, False)
    assert L.bcnf_fold_raw_table_bytes(ctypes.byref(no_an), 90, ctypes.byref(nb)) == N.ERR_UNSUPPORTED
    one = N.make_desc(19, [16] * 7, 1, 80, 0.1, True)
    assert L.bcnf_fold_raw_table_bytes(ctypes.byref(one), 90, ctypes.byref(nb)) == N.ERR_UNSUPPORTED
    fc = N.make_desc(19, [16] * 7, 32, 80, 0.1, True)
    assert L.bcnf_fold_raw_table_bytes(ctypes.byref(fc), 97, ctypes.byref(nb)) == N.ERR_UNSUPPORTED
    wide_c = N.make_desc(19, [16] * 7, 32, 129, 0.1, True)
    assert L.bcnf_fold_raw_table_bytes(ctypes.byref(wide_c), 90, ctypes.byref(nb)) == N.ERR_UNSUPPORTED


@pytest.mark.parametrize("shape", ["small", "fc_large"])
def test_wide_backward_plan_stays_inside_the_workspace(shape):
    """The host arithmetic of the folded wide backward's G-region split (bcnf_wide_backward_plan = what wide_backward
    computes before its launches; VERDICT r04 item 4 / r05 missing 3) at the batches where the feature side's split-K
    need crosses the region's size (small stack: between B = 34 and 35; FC_large: between 47 and 48), at B = 0 / 1 and
    at bench size, for the whole stack and single-block ranges, with and without dL/dx and [dWf | dbf]: G lies inside the
    training workspace that bcnf_wide_workspace_bytes reports, the tail (feature-side partials) inside G, and the
    range's parameter-gradient scratch inside G before the tail. tools/asan_host.sh runs this under AddressSanitizer."""
    from bcnf_amd import _native as N
    lib = N.lib()
    if shape == "small":     # tests/test_gpu_wide_ranges.py::_cfg_deep: nv 5, NH 3, HP 52, C 80, Xp 68
        d, nb, nv, xp = N.make_desc(19, [48] * 3, 5, 80, 0.2, True), 5, 5, 68
        Bs = [0, 1, 24, 33, 34, 35, 36, 47, 48, 77]
    else:                    # FC_large folded: X = 310 -> Xp = 312
        d, nb, nv, xp = N.make_desc(19, [526] * 5, 26, 1360, 0.407, True), 26, 26, 312
        Bs = [0, 1, 34, 35, 46, 47, 48, 49, 1024, 2048]
    out = (ctypes.c_int64 * 8)()
    for B in Bs:
        ws = N.query_i64(lib.bcnf_wide_workspace_bytes, ctypes.byref(d), ctypes.c_int64(B), ctypes.c_int32(1))
        crossed = set()
        for lo, hi in [(0, nb), (0, 1), (nb - 1, nb), (1, nb)]:
            for want_dx, want_dwfb in [(1, 1), (1, 0), (0, 1), (0, 0)]:
                rc = lib.bcnf_wide_backward_plan(ctypes.byref(d), B, xp, want_dx, want_dwfb, lo, hi, out)
                assert rc == N.OK
                total, goff, gfl, tail, gsc_off, gsc_fl, dxn, dwn = list(out)
                assert 4 * total == ws
                assert 0 <= goff and goff + gfl <= total
                assert 0 <= tail <= gfl and tail == max(dxn, dwn)
                assert 0 <= gsc_off and gsc_fl >= 0 and gsc_off + gsc_fl <= gfl - tail
                if lo > 0:
                    assert tail == 0
                full_dwfb = nv * 80 * xp if shape == "small" else nv * 1360 * xp
                if want_dwfb and lo == 0:
                    assert dwn == (full_dwfb if full_dwfb <= gfl else 0)
                    crossed.add(full_dwfb <= gfl)
                if want_dx and lo == 0:
                    assert dxn == (nv * B * xp if nv * B * xp <= gfl else 0)
        if shape == "small" and B in (34, 35):
            assert crossed == {B == 35}          # the [dWf | dbf] need stops fitting below B = 35
    assert lib.bcnf_wide_backward_plan(ctypes.byref(d), 8, xp, 1, 1, 0, nb + 1, out) == N.ERR_ARG
    assert lib.bcnf_wide_backward_plan(ctypes.byref(d), 8, xp, 1, 1, 2, 2, out) == N.ERR_ARG

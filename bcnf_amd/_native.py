"""ctypes binding of the C-ABI in include/bcnf_amd.h (libbcnf_amd.so, built for gfx950).

`import torch` happens first on purpose: torch ships its own libamdhip64.so.7; loading it before
our library makes the dynamic linker resolve our DT_NEEDED libamdhip64.so.7 to torch's copy, so the
HIP stream handles torch hands us belong to the same runtime.

There is no fallback: if the library is missing every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede loading the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BCNF_AMD_LIB") or os.path.join(_HERE, "libbcnf_amd.so")   # override: A/B experiments

MAX_HIDDEN = 8

OK, ERR_ARG, ERR_UNSUPPORTED, ERR_HIP = 0, 1, 2, 3
ERR_HIP_BASE = 1000          # include/bcnf_amd.h: BCNF_ERR_HIP_BASE + hipError_t

# Every symbol include/bcnf_amd.h declares (checked by tests/test_native_abi.py).
EXPORTS = (
    "bcnf_stack_supported", "bcnf_param_count", "bcnf_packed_bytes", "bcnf_workspace_bytes",
    "bcnf_slab_bytes", "bcnf_pack_params", "bcnf_stack_forward", "bcnf_stack_backward",
    "bcnf_stack_inverse", "bcnf_grad_reduce", "bcnf_status_string",
    "bcnf_nll_forward", "bcnf_nll_backward", "bcnf_grad_partials", "bcnf_adam_step", "bcnf_adam_step_bookkeep",
    "bcnf_grad_sumsq",
    "bcnf_clip_grad_norm", "bcnf_linear_forward", "bcnf_linear_work_bytes", "bcnf_linear_backward",
    "bcnf_linear_gelu_forward", "bcnf_linear_gelu_backward",
    "bcnf_inverse_scratch_bytes", "bcnf_stack_dh", "bcnf_backward_tail", "bcnf_gather_rows2",
    "bcnf_gather_batch", "bcnf_advance_counters", "bcnf_fold_bytes", "bcnf_fold_slab_bytes",
    "bcnf_pack_params_fold", "bcnf_fold_nll_forward", "bcnf_fold_backward_tail",
    "bcnf_fold_raw_table_bytes", "bcnf_fold_raw_table", "bcnf_fold_train_forward", "bcnf_lds_fill",
    "bcnf_wide_supported", "bcnf_wide_param_count", "bcnf_wide_packed_bytes", "bcnf_wide_workspace_bytes", "bcnf_wide_inverse_scratch_bytes",
    "bcnf_wide_pack", "bcnf_wide_forward", "bcnf_wide_nll_finalize", "bcnf_wide_backward", "bcnf_wide_inverse",
    "bcnf_wide_fold_prepare", "bcnf_wide_fold_forward", "bcnf_wide_fold_backward", "bcnf_wide_proj_rows",
    "bcnf_wide_fold_backward_range", "bcnf_wide_fold_backward_phase", "bcnf_wide_block_offset",
    "bcnf_wide_gemm_test", "bcnf_wide_backward_plan", "bcnf_rank_count", "bcnf_resimulate",
    "bcnf_guard_check_global", "bcnf_abi_version",
)
ABI_VERSION = 2          # include/bcnf_amd.h BCNF_AMD_ABI_VERSION (the struct layouts below)
MAX_TENSORS = 48


class BcnfStackDesc(ctypes.Structure):
    _fields_ = [
        ("size", ctypes.c_int32),
        ("n_conditions", ctypes.c_int32),
        ("n_hidden", ctypes.c_int32),
        ("hidden", ctypes.c_int32 * MAX_HIDDEN),
        ("n_blocks", ctypes.c_int32),
        ("act_norm", ctypes.c_int32),
        ("two_way", ctypes.c_int32),
        ("dropout", ctypes.c_float),
        ("gemm_tiling", ctypes.c_int32),      # wide family: 0 = cost model, t + 1 forces tiling t (per call)
    ]


class BcnfFoldAdam(ctypes.Structure):
    """include/bcnf_amd.h BcnfFoldAdam: Adam fused into bcnf_fold_backward_tail."""
    _fields_ = [
        ("params", ctypes.c_void_p * 3),
        ("exp_avg", ctypes.c_void_p * 3),
        ("exp_avg_sq", ctypes.c_void_p * 3),
        ("step", ctypes.c_void_p),
        ("lr", ctypes.c_double),
        ("beta1", ctypes.c_double),
        ("beta2", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("weight_decay", ctypes.c_double),
        ("advance_cursor", ctypes.c_void_p),
        ("cursor_modulo", ctypes.c_int64),
        ("log_values", ctypes.c_void_p),
        ("log_history", ctypes.c_void_p),
        ("done_counter", ctypes.c_void_p),
        ("guard", ctypes.c_void_p),
    ]


class BcnfGather2(ctypes.Structure):
    """include/bcnf_amd.h BcnfGather2: a batch gather run inside bcnf_pack_params_fold's launch."""
    _fields_ = [
        ("idx", ctypes.c_void_p),
        ("cursor", ctypes.c_void_p),
        ("n", ctypes.c_int64),
        ("src0", ctypes.c_void_p),
        ("cols0", ctypes.c_int32),
        ("dst0", ctypes.c_void_p),
        ("src1", ctypes.c_void_p),
        ("cols1", ctypes.c_int32),
        ("dst1", ctypes.c_void_p),
    ]


def make_desc(size, nested_sizes, n_blocks, n_conditions, dropout=0.0, act_norm=False, two_way=False):
    d = BcnfStackDesc()
    d.size = int(size)
    d.n_conditions = int(n_conditions)
    d.n_hidden = len(nested_sizes)
    if len(nested_sizes) > MAX_HIDDEN:
        raise ValueError(f"bcnf_amd supports at most {MAX_HIDDEN} nested layers, got {len(nested_sizes)}")
    for i, hsz in enumerate(nested_sizes):
        d.hidden[i] = int(hsz)
    d.n_blocks = int(n_blocks)
    d.act_norm = 1 if act_norm else 0
    d.two_way = 1 if two_way else 0
    d.dropout = float(dropout)
    return d


_lib = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_pdesc = ctypes.POINTER(BcnfStackDesc)
_pi64 = ctypes.POINTER(ctypes.c_int64)


def _bind(lib):
    sig = {
        "bcnf_stack_supported": (_i32, [_pdesc]),
        "bcnf_param_count": (_i32, [_pdesc, _pi64, _pi64]),
        "bcnf_packed_bytes": (_i32, [_pdesc, _pi64]),
        "bcnf_workspace_bytes": (_i32, [_pdesc, _i64, _i32, _pi64]),
        "bcnf_slab_bytes": (_i32, [_pdesc, _i64, _pi64]),
        "bcnf_pack_params": (_i32, [_pdesc, _vp, _vp, _vp, _vp]),
        "bcnf_inverse_scratch_bytes": (_i32, [_pdesc, _i64, _pi64]),
        "bcnf_stack_dh": (_i32, [_pdesc, _vp, _vp, _i64, _i32, _vp, _vp]),
        "bcnf_backward_tail": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp]),
        "bcnf_gather_rows2": (_i32, [_vp, _i64, _vp, _i32, _vp, _vp, _i32, _vp, _vp]),
        "bcnf_gather_batch": (_i32, [_vp, _vp, _i64, _vp, _i32, _vp, _vp, _i32, _vp, _vp]),
        "bcnf_advance_counters": (_i32, [_vp, _vp, _i64, _vp]),
        "bcnf_guard_check_global": (_i32, [_vp, _vp, _vp]),
        "bcnf_stack_forward": (_i32, [_pdesc, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _vp]),
        "bcnf_stack_backward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
        "bcnf_stack_inverse": (_i32, [_pdesc, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i32, _vp, _vp, _vp]),
        "bcnf_grad_reduce": (_i32, [_pdesc, _vp, _vp, _vp, _i64, _i32, _vp, _vp]),
        "bcnf_nll_forward": (_i32, [_pdesc, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp]),
        "bcnf_nll_backward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp]),
        "bcnf_fold_bytes": (_i32, [_pdesc, _i32, _pi64]),
        "bcnf_fold_slab_bytes": (_i32, [_pdesc, _i32, _i64, _pi64]),
        "bcnf_pack_params_fold": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
        "bcnf_fold_nll_forward": (_i32, [_pdesc, _vp, _vp, _i32, _vp, _vp, _i32, _i64, _vp, _vp, _i32, _vp, _vp,
                                         _i32, _vp, _vp, _vp]),
        "bcnf_fold_raw_table_bytes": (_i32, [_pdesc, _i32, _pi64]),
        "bcnf_lds_fill": (_i32, [ctypes.c_float, _vp]),
        "bcnf_fold_raw_table": (_i32, [_pdesc, _i32, _vp]),
        "bcnf_fold_train_forward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i64, _vp,
                                           _vp, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp]),
        "bcnf_fold_backward_tail": (_i32, [_pdesc, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _i64, _i32, _vp, _vp,
                                           _vp, _vp, _vp]),
        "bcnf_grad_partials": (_i64, [_i64]),
        "bcnf_adam_step": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_double, ctypes.c_double, _vp, _i32, _vp, _vp]),
        "bcnf_adam_step_bookkeep": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double, _vp, _i64, _vp, _vp,
                                           _vp, _vp, _vp]),
        "bcnf_grad_sumsq": (_i32, [_i32, _vp, _vp, _vp, _vp]),
        "bcnf_clip_grad_norm": (_i32, [_i32, _vp, _vp, _vp, ctypes.c_float, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                       _vp]),
        "bcnf_linear_forward": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp]),
        "bcnf_linear_work_bytes": (_i64, [_i64, _i32, _i32]),
        "bcnf_linear_backward": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
        "bcnf_linear_gelu_forward": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, ctypes.c_float, _vp, _i32, _vp, _vp,
                                            _vp]),
        "bcnf_linear_gelu_backward": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
        "bcnf_wide_supported": (_i32, [_pdesc]),
        "bcnf_wide_param_count": (_i32, [_pdesc, _pi64, _pi64]),
        "bcnf_wide_packed_bytes": (_i32, [_pdesc, _pi64]),
        "bcnf_wide_workspace_bytes": (_i32, [_pdesc, _i64, _i32, _pi64]),
        "bcnf_wide_inverse_scratch_bytes": (_i32, [_pdesc, _i64, _i64, _pi64]),
        "bcnf_wide_pack": (_i32, [_pdesc, _vp, _vp, _vp, _vp]),
        "bcnf_wide_forward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _vp]),
        "bcnf_wide_fold_prepare": (_i32, [_pdesc, _vp, _vp, _i32, _vp, _vp]),
        "bcnf_wide_fold_forward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _vp]),
        "bcnf_wide_fold_backward": (_i32, [_pdesc, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                           _vp, _vp]),
        "bcnf_wide_fold_backward_range": (_i32, [_pdesc, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                 _vp, _vp, _i32, _i32, _vp]),
        "bcnf_wide_fold_backward_phase": (_i32, [_pdesc, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                 _vp, _vp, _i32, _vp]),
        "bcnf_wide_block_offset": (_i32, [_pdesc, _i32, _pi64]),
        "bcnf_wide_proj_rows": (_i32, [_pdesc, _pi64]),
        "bcnf_wide_nll_finalize": (_i32, [_pdesc, _vp, _i64, _i32, _vp, _vp, _vp, _vp]),
        "bcnf_wide_backward": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _vp, _vp, _vp,
                                      _vp]),
        "bcnf_wide_inverse": (_i32, [_pdesc, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i32, _vp, _vp, _vp]),
        "bcnf_rank_count": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp]),
        "bcnf_resimulate": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _i32, ctypes.c_double, _i32,
                                   ctypes.c_double, ctypes.c_double, _i32, _vp, _vp, _vp, _vp]),
        "bcnf_wide_gemm_test": (_i32, [_i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp]),
        "bcnf_wide_backward_plan": (_i32, [_pdesc, _i64, _i32, _i32, _i32, _i32, _i32, _pi64]),
        "bcnf_status_string": (ctypes.c_char_p, [_i32]),
        "bcnf_abi_version": (_i32, []),
    }
    override = "BCNF_AMD_LIB" in os.environ     # an explicit A/B build (tools/): it may predate newer entry points
    for name, (res, args) in sig.items():
        if override and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """The loaded HIP library. Raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"bcnf_amd: HIP library {LIB_PATH} is missing. Build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950).")
                handle = ctypes.CDLL(LIB_PATH)
                _bind(handle)
                if (hasattr(handle, "bcnf_abi_version") or "BCNF_AMD_LIB" not in os.environ) and \
                        handle.bcnf_abi_version() != ABI_VERSION:
                    raise RuntimeError(f"bcnf_amd: {LIB_PATH} has ABI version {handle.bcnf_abi_version()}, the "
                                       f"bindings expect {ABI_VERSION}: rebuild the library")
                _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != OK:
        L = lib()
        msg = L.bcnf_status_string(rc).decode()
        extra = f" (hipError {rc - ERR_HIP_BASE})" if rc >= ERR_HIP_BASE else ""
        raise RuntimeError(f"bcnf_amd: {what} failed: {msg}{extra}")


def ptr(t):
    return ctypes.c_void_p(0) if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr_array(tensors):
    """ctypes array of device pointers (None -> NULL) for the multi-tensor entry points."""
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def i64_array(values):
    arr = (ctypes.c_int64 * len(values))()
    for i, v in enumerate(values):
        arr[i] = int(v)
    return arr


def query_i64(fn, *args) -> int:
    out = ctypes.c_int64(0)
    check(fn(*args, ctypes.byref(out)), fn.__name__)
    return int(out.value)

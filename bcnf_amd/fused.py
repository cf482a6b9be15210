"""Host runtime of the fused HIP coupling stack: flat parameter storage, packing, workspaces and the
autograd boundary. PyTorch provides device memory, streams and autograd plumbing; all arithmetic of
the coupling stack runs in libbcnf_amd.so (bcnf_amd/csrc/bcnf_stack.hip).

Parameter storage
-----------------
The trainable coupling-stack parameters (ActNorm scale/bias + every nested-MLP Linear, in state_dict
order, orthonormal matrices excluded) live in ONE contiguous fp32 buffer; every nn.Parameter of the
reference module tree (`layers.0.scale`, `layers.1.nn_a.nn.0.weight`, ...) is a view into it, so
state_dict / load_state_dict / optimizers keep working unchanged. The frozen orthonormal matrices
live in a second buffer. `flat_param` is a leaf Parameter over the same storage: the autograd
Function returns the whole flat gradient for it in a single AccumulateGrad. In "per_param" grad mode
(the default, what the unchanged bcnf Trainer expects) a post-accumulate hook additionally exposes
per-layer `.grad` tensors as views of that flat gradient.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

from bcnf_amd import _native as N


@dataclass
class StackConfig:
    size: int
    nested_sizes: tuple
    n_blocks: int
    n_conditions: int
    dropout: float
    act_norm: bool
    two_way: bool

    def desc(self):
        return N.make_desc(self.size, list(self.nested_sizes), self.n_blocks, self.n_conditions, self.dropout,
                           self.act_norm, self.two_way)


class FusedStack:
    """Owns the flat parameter buffers of one coupling stack and drives the HIP kernels."""

    def __init__(self, cfg: StackConfig, trainable: list, frozen: list, bind: bool = True):
        self.cfg = cfg
        self.bind = bind
        self.desc = cfg.desc()
        self._pdesc = ctypes.byref(self.desc)
        self.trainable = list(trainable)   # canonical order (state_dict order, orthonormal excluded)
        self.frozen = list(frozen)         # orthonormal matrices, block order
        self.grad_mode = "per_param"
        self._packed = None
        self._pack_frozen = False
        self._rng_state = None
        self.seed = None
        self.timers = None       # dict -> per-kernel HIP-event pairs (bench.py kernel timing phase)
        self.guard = None        # device int32[BCNF_GUARD_WORDS] divergence guard of a TrainStep, or None
        if bind:
            self.flatten()
        else:   # standalone layer: flat params are provided per call (see stack_forward(flat=...))
            self.flat = None
            self.qflat = None
            self.flat_param = None

    # ------------------------------------------------------------------ layout
    @property
    def supported(self) -> bool:
        return bool(N.lib().bcnf_stack_supported(self._pdesc))

    def counts(self):
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(N.lib().bcnf_param_count(self._pdesc, ctypes.byref(a), ctypes.byref(b)), "bcnf_param_count")
        return int(a.value), int(b.value)

    def flatten(self):
        """(Re)build the flat buffers on the parameters' current device and rebind every Parameter
        to a view of them. Called at construction and after every Module._apply (to(), cuda(), ...)."""
        params = self.trainable
        dev = params[0].device
        n = sum(p.numel() for p in params)
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + k].view(p.shape)
                off += k
        nq = sum(q.numel() for q in self.frozen)
        qflat = torch.empty(max(nq, 1), dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for q in self.frozen:
                k = q.numel()
                qflat[off:off + k].copy_(q.detach().reshape(-1))
                q.data = qflat[off:off + k].view(q.shape)
                off += k
        self.flat = flat
        self.qflat = qflat
        self.flat_param = torch.nn.Parameter(flat, requires_grad=True)
        self.flat_param.register_post_accumulate_grad_hook(self._on_flat_grad)
        self._offsets = []
        off = 0
        for p in params:
            self._offsets.append((off, p.numel()))
            off += p.numel()
        self._packed = None
        self._rng_state = None
        self._raw_tables = {}

    def _on_flat_grad(self, fp):
        if self.grad_mode != "per_param" or fp.grad is None:
            return
        g = fp.grad
        for p, (off, k) in zip(self.trainable, self._offsets):
            p.grad = g[off:off + k].view(p.shape)

    def sync_grad_state(self):
        """The Trainer zeroes per-layer grads (set_to_none); drop the stale flat grad with them."""
        if self.bind and self.grad_mode == "per_param" and self.trainable[0].grad is None:
            self.flat_param.grad = None

    # ------------------------------------------------------------------ device helpers
    def _check_inputs(self, x, h, what):
        cfg = self.cfg
        if x.dim() != 2 or x.shape[1] != cfg.size:
            raise ValueError(f"bcnf_amd {what}: expected (N, {cfg.size}) input, got {tuple(x.shape)}")
        if h.dim() != 2 or h.shape[1] != cfg.n_conditions:
            raise ValueError(f"bcnf_amd {what}: expected features (N, {cfg.n_conditions}), got {tuple(h.shape)}")
        self._check_device(x, h)

    def _check_device(self, *tensors):
        for t in tensors:
            if t is None:
                continue
            if not t.is_cuda:
                raise RuntimeError("bcnf_amd runs the coupling stack on the MI355X HIP kernels only; "
                                   "move the model and inputs to a ROCm device (model.to('cuda')).")
            if t.dtype != torch.float32:
                raise TypeError(f"bcnf_amd coupling stack is fp32-only, got {t.dtype}")
        if self.flat is None or self.flat.device.type != "cuda":
            raise RuntimeError("bcnf_amd: model parameters are not on the GPU; call model.to('cuda') first.")

    def packed(self, fresh: bool = False):
        """Packed LDS-record buffer. Re-packed on every call unless inside `reuse_pack()` (parameters
        change in place after each optimizer step; `.data`-rebound views do not share one reliable
        version counter, so no staleness heuristics). Under HIP-graph capture the pack is a graph node."""
        if fresh and not self._pack_frozen:
            # private copy that a later forward cannot overwrite before this one's backward runs
            nbytes = N.query_i64(N.lib().bcnf_packed_bytes, self._pdesc)
            out = torch.empty(nbytes // 4, dtype=torch.float32, device=self.flat.device)
            self._pack_into(out)
            return out
        if self._packed is None:
            nbytes = N.query_i64(N.lib().bcnf_packed_bytes, self._pdesc)
            self._packed = torch.empty(nbytes // 4, dtype=torch.float32, device=self.flat.device)
        if not self._pack_frozen:
            self._pack_into(self._packed)
        return self._packed

    def _pack_into(self, out):
        rc = N.lib().bcnf_pack_params(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(out),
                                      N.stream_handle(self.flat.device))
        N.check(rc, "bcnf_pack_params")

    class _Reuse:
        def __init__(self, stack):
            self.stack = stack

        def __enter__(self):
            self.stack.packed()
            self.prev = self.stack._pack_frozen
            self.stack._pack_frozen = True
            return self.stack

        def __exit__(self, *exc):
            self.stack._pack_frozen = self.prev

    def reuse_pack(self):
        """Pack once and reuse it for every launch inside the block (e.g. all chunks of sample())."""
        return FusedStack._Reuse(self)

    # A feature network bound to this stack draws its dropout from the same (seed, offset) and leaves the advance to
    # the coupling launch that follows in the step (feature_network.py). True between such a feature draw and the
    # next coupling launch: a second feature draw before any coupling launch (the feature network run on its own)
    # advances the offset itself first (feature_rng_state), so repeated standalone calls draw fresh masks.
    _feature_pending = False

    def rng_state(self):
        """Device-resident (seed, offset) for the in-kernel Philox dropout; the offset is bumped by a
        device-side add after every training forward, so HIP-graph replays draw fresh masks."""
        self._feature_pending = False          # a coupling launch takes this step's offset
        return self._rng_tensor()

    def feature_rng_state(self):
        """The state a bound feature network's fused dropout draws from, when the coupling launch of the step will
        advance it (a feature draw not followed by a coupling launch advances it at the next one)."""
        t = self._rng_tensor()
        if self._feature_pending:
            t[1:2].add_(1)
        self._feature_pending = True
        return t

    def _rng_tensor(self):
        if self._rng_state is None:
            seed = self.seed
            if seed is None:
                seed = (torch.cuda.initial_seed() * 0x9E3779B97F4A7C15 + id(self)) & ((1 << 62) - 1)
            self._rng_state = torch.tensor([seed, 0], dtype=torch.int64, device=self.flat.device)
        return self._rng_state

    def set_seed(self, seed: int):
        self.seed = int(seed)
        self._rng_state = None

    def workspace_bytes(self, batch: int, training: bool):
        L = N.lib()
        wb = N.query_i64(L.bcnf_workspace_bytes, self._pdesc, ctypes.c_int64(batch), ctypes.c_int32(int(training)))
        sb = N.query_i64(L.bcnf_slab_bytes, self._pdesc, ctypes.c_int64(batch))
        return wb, sb

    # ------------------------------------------------------------------ launches
    def launch_forward(self, y, h, training: bool, save: bool, want_logp: bool = False):
        self._check_inputs(y, h, "forward")
        if h.shape[0] != y.shape[0]:
            raise ValueError(f"bcnf_amd forward: {y.shape[0]} samples but {h.shape[0]} feature rows")
        B = y.shape[0]
        dev = y.device
        z = torch.empty_like(y)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        logp = torch.empty(B, dtype=torch.float32, device=dev) if want_logp else None
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        wb, _ = self.workspace_bytes(B, training)      # also holds the condition projection
        ws = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
        pk = self.packed(fresh=save)
        tm = self.timers
        if tm is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        rc = N.lib().bcnf_stack_forward(self._pdesc, N.ptr(pk), N.ptr(y), N.ptr(h), ctypes.c_int64(B), N.ptr(z),
                                        N.ptr(ldj), N.ptr(logp), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                                        ctypes.c_int32(int(save)), N.stream_handle(dev))
        N.check(rc, "bcnf_stack_forward")
        if tm is not None:
            e1.record()
            tm.setdefault("k_forward", []).append((e0, e1))
        if drop:
            rng[1:2].add_(1)
        return z, ldj, logp, (ws, pk)

    def launch_backward(self, h, dz, dldj, training: bool, saved, want_dy: bool, want_dh: bool):
        ws, pk = saved
        B = h.shape[0]
        dev = h.device
        _, sb = self.workspace_bytes(B, training)
        slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty_like(self.flat)
        dh = torch.empty_like(h) if want_dh else None
        dy = torch.empty((B, self.cfg.size), dtype=torch.float32, device=dev) if want_dy else None
        stream = N.stream_handle(dev)
        tm = self.timers
        e0 = None
        if tm is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        rc = N.lib().bcnf_stack_backward(self._pdesc, N.ptr(pk), N.ptr(h), N.ptr(dz), N.ptr(dldj),
                                         ctypes.c_int64(B), ctypes.c_int32(int(training)), N.ptr(ws), N.ptr(dy),
                                         None, None, N.ptr(slab), stream)
        N.check(rc, "bcnf_stack_backward")
        self._backward_tail(h, ws, pk, slab, dh, dparams, B, training, stream, tm, e0)
        return dy, dh, dparams

    def _backward_tail(self, h, ws, pk, slab, dh, dparams, B, training, stream, tm, e0):
        """dL/dh and the deterministic parameter-gradient reduction after a backward launch (one fused tail
        launch + the split-K finish); with timers, the backward and the tail get HIP-event pairs."""
        if tm is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            tm.setdefault("k_backward", []).append((e0, e1))
            e0 = e1
        N.check(N.lib().bcnf_backward_tail(self._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(h), N.ptr(ws), ctypes.c_int64(B),
                                           ctypes.c_int32(int(training)), N.ptr(dh), N.ptr(dparams), stream),
                "bcnf_backward_tail")
        if tm is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            tm.setdefault("k_bwd_tail", []).append((e0, e1))

    def launch_nll_forward(self, y, h, training: bool, finalize: bool = True):
        """Stack forward fused with inn_nll_loss (trainer.py:260-266): returns z, ldj, vals=[loss, nll, mse]
        and the saved state for launch_nll_backward. With finalize=False the loss reduction and the
        dropout-RNG advance are deferred to the backward (vals is valid only after it)."""
        self._check_inputs(y, h, "forward")
        if h.shape[0] != y.shape[0]:
            raise ValueError(f"bcnf_amd forward: {y.shape[0]} samples but {h.shape[0]} feature rows")
        B = y.shape[0]
        if B == 0:
            raise ValueError("bcnf_amd: the NLL of an empty batch is undefined")
        dev = y.device
        z = torch.empty_like(y)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        vals = torch.empty(3, dtype=torch.float32, device=dev)
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        wb, _ = self.workspace_bytes(B, training)
        ws = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
        pk = self.packed(fresh=True)
        tm = self.timers
        if tm is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        rc = N.lib().bcnf_nll_forward(self._pdesc, N.ptr(pk), N.ptr(y), N.ptr(h), ctypes.c_int64(B), N.ptr(z),
                                      N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                                      ctypes.c_int32(int(finalize)), N.ptr(vals), N.ptr(self.guard if finalize else None),
                                      N.stream_handle(dev))
        N.check(rc, "bcnf_nll_forward")
        if tm is not None:
            e1.record()
            tm.setdefault("k_forward", []).append((e0, e1))
        return z, ldj, vals, (ws, pk)

    def launch_nll_backward(self, h, z, dvals, training: bool, saved, want_dy: bool, want_dh: bool,
                            finalize_into=None):
        ws, pk = saved
        B = h.shape[0]
        dev = h.device
        _, sb = self.workspace_bytes(B, training)
        slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty_like(self.flat)
        dh = torch.empty_like(h) if want_dh else None
        dy = torch.empty((B, self.cfg.size), dtype=torch.float32, device=dev) if want_dy else None
        stream = N.stream_handle(dev)
        tm = self.timers
        e0 = None
        if tm is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        rng = self.rng_state() if (finalize_into is not None and training and self.cfg.dropout > 0.0) else None
        rc = N.lib().bcnf_nll_backward(self._pdesc, N.ptr(pk), N.ptr(h), N.ptr(z), N.ptr(dvals), ctypes.c_int64(B),
                                       ctypes.c_int32(int(training)), N.ptr(ws), N.ptr(dy), None, None,
                                       N.ptr(slab), N.ptr(finalize_into), N.ptr(rng),
                                       N.ptr(self.guard if finalize_into is not None else None), stream)
        N.check(rc, "bcnf_nll_backward")
        self._backward_tail(h, ws, pk, slab, dh, dparams, B, training, stream, tm, e0)
        return dy, dh, dparams

    # ------------------------------------------------------------------ folded linear feature network
    def fold_supported(self, in_features: int) -> bool:
        """Whether a single nn.Linear [in_features -> n_conditions] feature network can be folded into the
        condition projection (bcnf_pack_params_fold; include/bcnf_amd.h)."""
        out = ctypes.c_int64(0)
        return N.lib().bcnf_fold_bytes(self._pdesc, ctypes.c_int32(int(in_features)), ctypes.byref(out)) == N.OK

    # bcnf_fold_train_forward (the pack-free folded forward, one launch) where its table applies; False: always the
    # two-launch form (pack + fold, then the forward) -- BCNF_FOLD_RAW=0 in the environment, for A/B runs
    use_raw_forward = os.environ.get("BCNF_FOLD_RAW", "1") != "0"

    def raw_table(self, X: int):
        """The device copy of bcnf_fold_raw_table for in_features X (built once per device), or None where the
        pack-free forward does not apply (or the library predates it)."""
        if not self.use_raw_forward or not hasattr(N.lib(), "bcnf_fold_train_forward"):
            return None
        dev = self.flat.device
        key = (X, str(dev))
        if key not in self._raw_tables:
            if torch.cuda.is_current_stream_capturing():
                return None                     # no host -> device copy inside a graph capture
            L = N.lib()
            nb = ctypes.c_int64(0)
            if L.bcnf_fold_raw_table_bytes(self._pdesc, ctypes.c_int32(X), ctypes.byref(nb)) != N.OK:
                self._raw_tables[key] = None
            else:
                host = torch.empty(nb.value // 4, dtype=torch.int32)
                N.check(L.bcnf_fold_raw_table(self._pdesc, ctypes.c_int32(X), ctypes.c_void_p(host.data_ptr())),
                        "bcnf_fold_raw_table")
                self._raw_tables[key] = host.to(dev)
        return self._raw_tables[key]

    def launch_fold_nll_forward(self, y, x, wf, bf, training: bool, finalize: bool = True, gather=None):
        """launch_nll_forward with h = x Wf^T + bf never formed as a tensor. Pack-free form (raw_table applies):
        ONE launch, bcnf_fold_train_forward, builds its records from the parameters and computes h of its rows
        on the fly. Otherwise the pack launch also folds the Linear into the projection weights (Wc = W1h Wf,
        bc = b1 + W1h bf) and the projection runs on x. gather (an N.BcnfGather2 that fills y and x): the batch
        gather runs inside the first launch."""
        self._check_device(y, x, wf, bf)
        B, X = x.shape
        if y.dim() != 2 or y.shape != (B, self.cfg.size):
            raise ValueError(f"bcnf_amd folded forward: y {tuple(y.shape)} vs x {tuple(x.shape)}")
        if B == 0:
            raise ValueError("bcnf_amd: the NLL of an empty batch is undefined")
        L = N.lib()
        dev = y.device
        stream = N.stream_handle(dev)
        pk = torch.empty(N.query_i64(L.bcnf_packed_bytes, self._pdesc) // 4, dtype=torch.float32, device=dev)
        table = self.raw_table(X)
        if table is not None:
            z = torch.empty_like(y)
            ldj = torch.empty(B, dtype=torch.float32, device=dev)
            vals = torch.empty(3, dtype=torch.float32, device=dev)
            rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
            wb, _ = self.workspace_bytes(B, training)
            ws = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
            rc = L.bcnf_fold_train_forward(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(table), N.ptr(wf),
                                           N.ptr(bf), ctypes.c_int32(X),
                                           None if gather is None else ctypes.byref(gather), N.ptr(y), N.ptr(x),
                                           ctypes.c_int32(x.stride(0)), ctypes.c_int64(B), N.ptr(pk), N.ptr(z),
                                           N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                                           ctypes.c_int32(int(finalize)), N.ptr(vals),
                                           N.ptr(self.guard if finalize else None), stream)
            N.check(rc, "bcnf_fold_train_forward")
            return z, ldj, vals, (ws, pk)
        fold = torch.empty(N.query_i64(L.bcnf_fold_bytes, self._pdesc, ctypes.c_int32(X)) // 4, dtype=torch.float32,
                           device=dev)
        N.check(L.bcnf_pack_params_fold(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(wf), N.ptr(bf),
                                        ctypes.c_int32(X), N.ptr(pk), N.ptr(fold),
                                        None if gather is None else ctypes.byref(gather), stream),
                "bcnf_pack_params_fold")
        z = torch.empty_like(y)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        vals = torch.empty(3, dtype=torch.float32, device=dev)
        rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
        wb, _ = self.workspace_bytes(B, training)
        ws = torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)
        rc = L.bcnf_fold_nll_forward(self._pdesc, N.ptr(pk), N.ptr(fold), ctypes.c_int32(X), N.ptr(y), N.ptr(x),
                                     ctypes.c_int32(x.stride(0)), ctypes.c_int64(B), N.ptr(z), N.ptr(ldj), ctypes.c_int32(int(training)),
                                     N.ptr(rng), N.ptr(ws), ctypes.c_int32(int(finalize)), N.ptr(vals),
                                     N.ptr(self.guard if finalize else None), stream)
        N.check(rc, "bcnf_fold_nll_forward")
        return z, ldj, vals, (ws, pk)

    # A BcnfFoldAdam for the next folded backward (TrainStep, multi-step graphs): consumed by that launch.
    pending_adam = None
    # (bucket, (flat offset, feature W offset, feature b offset)): TrainStep's data-parallel gradient bucket, which
    # the folded backward writes its gradients into.
    grad_bucket = None

    def launch_fold_nll_backward(self, x, z, dvals, wf, bf, training: bool, saved, want_feat: bool,
                                 finalize_into=None, adam=None):
        """Fused NLL backward of the folded pass: (dparams, dWf, dbf); no dL/dh, no dL/dx. adam (an
        N.BcnfFoldAdam): the optimizer update of every parameter runs inside the backward tail."""
        ws, pk = saved
        B, X = x.shape
        L = N.lib()
        dev = x.device
        stream = N.stream_handle(dev)
        sb = N.query_i64(L.bcnf_fold_slab_bytes, self._pdesc, ctypes.c_int32(X), ctypes.c_int64(B))
        slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=dev)
        gb = self.grad_bucket
        if gb is not None and want_feat:
            # data parallel (TrainStep): the gradients land in the all-reduce bucket itself, as fresh views that
            # autograd adopts as .grad, so no bucket copy follows the backward
            bucket, offs = gb
            dparams = bucket.narrow(0, offs[0], self.flat.numel()).view_as(self.flat)
            dwf = bucket.narrow(0, offs[1], wf.numel()).view_as(wf)
            dbf = bucket.narrow(0, offs[2], bf.numel()).view_as(bf) if bf is not None else None
        else:
            dparams = torch.empty_like(self.flat)
            dwf = torch.empty_like(wf) if want_feat else None
            dbf = torch.empty_like(bf) if (want_feat and bf is not None) else None
        rng = self.rng_state() if (finalize_into is not None and training and self.cfg.dropout > 0.0) else None
        rc = L.bcnf_nll_backward(self._pdesc, N.ptr(pk), N.ptr(x), N.ptr(z), N.ptr(dvals), ctypes.c_int64(B),
                                 ctypes.c_int32(int(training)), N.ptr(ws), None, None, None, N.ptr(slab),
                                 N.ptr(finalize_into), N.ptr(rng),
                                 N.ptr(self.guard if finalize_into is not None else None), stream)
        N.check(rc, "bcnf_nll_backward")
        N.check(L.bcnf_fold_backward_tail(self._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(x), ctypes.c_int32(x.stride(0)),
                                          ctypes.c_int32(X), N.ptr(wf),
                                          N.ptr(bf), N.ptr(ws), ctypes.c_int64(B), ctypes.c_int32(int(training)),
                                          N.ptr(dparams), N.ptr(dwf), N.ptr(dbf),
                                          None if adam is None else ctypes.byref(adam), stream),
                "bcnf_fold_backward_tail")
        return dparams, dwf, dbf

    @torch.no_grad()
    def time_kernels(self, y, h, training: bool = True, iters: int = 20, fold=None):
        """Average device time (us) of each launch of one NLL training pass, measured with HIP events on the
        launch stream around `iters` back-to-back launches of the same (idempotent) call, so host launch
        latency is amortised: 'forward' (k_hp + k_forward), 'k_backward' (the backward kernel alone) and
        'tail' (dh + slab reduce + W1 condition part). fold = (x, Wf, bf): the folded path instead -- 'pack'
        (pack + fold), 'forward' (k_hp on x + k_forward), 'k_backward', 'tail' (slab reduce + split-K on x,
        Gx reduce, dW1h / dWf / dbf)."""
        if fold is not None:
            return self._time_fold_kernels(y, *fold, training=training, iters=iters)
        L = N.lib()
        dev = y.device
        stream = N.stream_handle(dev)
        B = y.shape[0]
        z, _, vals, (ws, pk) = self.launch_nll_forward(y, h, training, finalize=False)
        _, sb = self.workspace_bytes(B, training)
        slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=dev)
        dh = torch.empty_like(h)
        dparams = torch.empty_like(self.flat)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
        calls = {
            "k_forward": lambda: L.bcnf_nll_forward(self._pdesc, N.ptr(pk), N.ptr(y), N.ptr(h), ctypes.c_int64(B), N.ptr(z),
                                                  N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                                                  ctypes.c_int32(0), N.ptr(vals), None, stream),
            "k_backward": lambda: L.bcnf_nll_backward(self._pdesc, N.ptr(pk), N.ptr(h), N.ptr(z), None, ctypes.c_int64(B),
                                                      ctypes.c_int32(int(training)), N.ptr(ws), None, None, None,
                                                      N.ptr(slab), None, None, None, stream),
            "tail": lambda: L.bcnf_backward_tail(self._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(h), N.ptr(ws),
                                                 ctypes.c_int64(B), ctypes.c_int32(int(training)), N.ptr(dh),
                                                 N.ptr(dparams), stream),
        }
        return self._event_times(calls, iters)

    @staticmethod
    def _event_times(calls, iters):
        out = {}
        for name, fn in calls.items():
            N.check(fn(), name)                       # warm (code object, LDS attributes)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) * 1e3 / iters
        return out

    def _time_fold_kernels(self, y, x, wf, bf, training: bool, iters: int):
        L = N.lib()
        dev = y.device
        stream = N.stream_handle(dev)
        B, X = x.shape
        ldx = ctypes.c_int32(x.stride(0))
        z, _, vals, (ws, pk) = self.launch_fold_nll_forward(y, x, wf, bf, training, finalize=False)
        fold = torch.empty(N.query_i64(L.bcnf_fold_bytes, self._pdesc, ctypes.c_int32(X)) // 4, dtype=torch.float32,
                           device=dev)
        N.check(L.bcnf_pack_params_fold(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(wf), N.ptr(bf),
                                        ctypes.c_int32(X), N.ptr(pk), N.ptr(fold), None, stream), "pack_fold")
        sb = N.query_i64(L.bcnf_fold_slab_bytes, self._pdesc, ctypes.c_int32(X), ctypes.c_int64(B))
        slab = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty_like(self.flat)
        dwf, dbf = torch.empty_like(wf), (torch.empty_like(bf) if bf is not None else None)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
        table = self.raw_table(X)
        calls = {
            "k_pack_fold": lambda: L.bcnf_pack_params_fold(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(wf),
                                                    N.ptr(bf), ctypes.c_int32(X), N.ptr(pk), N.ptr(fold), None, stream),
            "k_forward": lambda: L.bcnf_fold_nll_forward(self._pdesc, N.ptr(pk), N.ptr(fold), ctypes.c_int32(X),
                                                       N.ptr(y), N.ptr(x), ldx, ctypes.c_int64(B), N.ptr(z),
                                                       N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng),
                                                       N.ptr(ws), ctypes.c_int32(0), N.ptr(vals), None, stream),
            "k_backward": lambda: L.bcnf_nll_backward(self._pdesc, N.ptr(pk), N.ptr(x), N.ptr(z), None,
                                                      ctypes.c_int64(B), ctypes.c_int32(int(training)), N.ptr(ws),
                                                      None, None, None, N.ptr(slab), None, None, None, stream),
            "tail": lambda: L.bcnf_fold_backward_tail(self._pdesc, N.ptr(pk), N.ptr(slab), N.ptr(x), ldx,
                                                      ctypes.c_int32(X), N.ptr(wf), N.ptr(bf), N.ptr(ws),
                                                      ctypes.c_int64(B), ctypes.c_int32(int(training)),
                                                      N.ptr(dparams), N.ptr(dwf), N.ptr(dbf), None, stream),
        }
        if table is not None:           # the pack-free forward: no pack launch
            del calls["k_pack_fold"]
            calls["k_forward"] = lambda: L.bcnf_fold_train_forward(
                self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(table), N.ptr(wf), N.ptr(bf), ctypes.c_int32(X),
                None, N.ptr(y), N.ptr(x), ldx, ctypes.c_int64(B), N.ptr(pk), N.ptr(z), N.ptr(ldj),
                ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws), ctypes.c_int32(0), N.ptr(vals), None, stream)
        return self._event_times(calls, iters)

    def launch_inverse(self, z, h, cond_index=None, training: bool = False):
        self._check_inputs(z, h, "inverse")
        n = z.shape[0]
        if cond_index is None and h.shape[0] != n:
            raise ValueError(f"bcnf_amd inverse: {n} latents but {h.shape[0]} feature rows and no cond_index")
        y = torch.empty_like(z)
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        if cond_index is not None:
            cond_index = cond_index.to(device=z.device, dtype=torch.int64).contiguous()
        hr = h.shape[0]
        sb = N.query_i64(N.lib().bcnf_inverse_scratch_bytes, self._pdesc, ctypes.c_int64(hr))
        scratch = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=z.device)
        rc = N.lib().bcnf_stack_inverse(self._pdesc, N.ptr(self.packed()), N.ptr(z), N.ptr(h), ctypes.c_int64(hr),
                                        N.ptr(cond_index), ctypes.c_int64(n), N.ptr(y), ctypes.c_int32(int(training)),
                                        N.ptr(rng), N.ptr(scratch), N.stream_handle(z.device))
        N.check(rc, "bcnf_stack_inverse")
        if drop:
            rng[1:2].add_(1)
        return y


class _StackForward(torch.autograd.Function):
    """z, ldj = stack(y, h). Backward runs the fused HIP backward once and returns dL/dy, dL/dh and the
    whole flat parameter gradient (one AccumulateGrad for `flat_param`)."""

    @staticmethod
    def forward(ctx, y, h, flat_param, stack: FusedStack, training: bool):
        needs = ctx.needs_input_grad
        save = any(needs[:3])
        z, ldj, _, saved = stack.launch_forward(y, h, training, save=save)
        ctx.stack = stack
        ctx.training = training
        ctx.saved = saved
        ctx.save_for_backward(h)
        return z, ldj

    @staticmethod
    def backward(ctx, dz, dldj):
        (h,) = ctx.saved_tensors
        stack = ctx.stack
        if dz is not None:
            dz = dz.contiguous()
        if dldj is not None:
            dldj = dldj.contiguous()
        need_y, need_h, need_p = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        dy, dh, dparams = stack.launch_backward(h, dz, dldj, ctx.training, ctx.saved, want_dy=need_y, want_dh=need_h)
        return dy, dh, (dparams if need_p else None), None, None


class _StackNLL(torch.autograd.Function):
    """vals = [loss, nll, mse] of inn_nll_loss(stack(y, h)) in one fused launch; backward is the fused NLL
    backward (no dz / dldj tensors, no elementwise loss kernels)."""

    @staticmethod
    def forward(ctx, y, h, flat_param, stack: FusedStack, training: bool, defer: bool):
        z, _, vals, saved = stack.launch_nll_forward(y, h, training, finalize=not defer)
        ctx.stack = stack
        ctx.training = training
        ctx.saved = saved
        ctx.defer = defer
        ctx.save_for_backward(h, z, vals)
        return vals

    @staticmethod
    def backward(ctx, dvals):
        h, z, vals = ctx.saved_tensors
        need_y, need_h, need_p = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        dy, dh, dparams = ctx.stack.launch_nll_backward(h, z, dvals.contiguous(), ctx.training, ctx.saved,
                                                        want_dy=need_y, want_dh=need_h,
                                                        finalize_into=vals if ctx.defer else None)
        return dy, dh, (dparams if need_p else None), None, None, None


def stack_nll(stack: FusedStack, y, h, training: bool, defer: bool = False):
    """[loss, nll, mse] (mse = 0, hybrid_weight = 0) of the Trainer's loss on the fused stack. defer=True
    (for a backward that certainly follows, e.g. TrainStep) lets the backward do the loss reduction and
    the dropout-RNG advance: one launch less, but vals is only valid after the backward."""
    y = y.contiguous()
    h = h.contiguous()
    stack.sync_grad_state()
    params_grad = stack.trainable[0].requires_grad
    fp = stack.flat_param
    if torch.is_grad_enabled() and (params_grad or y.requires_grad or h.requires_grad):
        return _StackNLL.apply(y, h, fp if params_grad else fp.detach(), stack, training, defer)
    return stack.launch_nll_forward(y, h, training)[2]


class _FoldNLL(torch.autograd.Function):
    """_StackNLL with the feature network's single nn.Linear folded into the condition projection: inputs
    (y, x, Wf, bf, flat_param); gradients for Wf, bf and flat_param (not for y or x)."""

    @staticmethod
    def forward(ctx, y, x, wf, bf, flat_param, stack: FusedStack, training: bool, defer: bool, gather):
        z, _, vals, saved = stack.launch_fold_nll_forward(y, x, wf, bf, training, finalize=not defer, gather=gather)
        ctx.stack = stack
        ctx.training = training
        ctx.saved = saved
        ctx.defer = defer
        ctx.save_for_backward(x, wf, bf, z, vals)
        return vals

    @staticmethod
    def backward(ctx, dvals):
        x, wf, bf, z, vals = ctx.saved_tensors
        need = ctx.needs_input_grad
        adam, ctx.stack.pending_adam = ctx.stack.pending_adam, None
        dparams, dwf, dbf = ctx.stack.launch_fold_nll_backward(x, z, dvals.contiguous(), wf, bf, ctx.training,
                                                               ctx.saved, want_feat=need[2] or need[3] or
                                                               adam is not None,
                                                               finalize_into=vals if ctx.defer else None, adam=adam)
        return (None, None, dwf if need[2] else None, dbf if need[3] else None, dparams if need[4] else None,
                None, None, None, None)


def stack_nll_fold(stack: FusedStack, y, x, wf, bf, training: bool, defer: bool = False, gather=None):
    """stack_nll(stack, y, x Wf^T + bf) without forming the features (see launch_fold_nll_forward). gather: the
    batch gather that fills y and x, run inside the pack launch (TrainStep); y and x are then its outputs."""
    if gather is not None and not (y.is_contiguous() and x.stride(1) == 1):
        raise ValueError("bcnf_amd: a deferred gather needs its own (contiguous) output buffers")
    y = y.contiguous()
    if x.stride(1) != 1 or x.stride(0) < x.shape[1]:
        x = x.contiguous()              # rows may be padded (ldx = stride(0) > X: TrainStep's zero-padded pool)
    stack.sync_grad_state()
    params_grad = stack.trainable[0].requires_grad
    fp = stack.flat_param
    feat_grad = wf.requires_grad or (bf is not None and bf.requires_grad)
    if torch.is_grad_enabled() and (params_grad or feat_grad):
        return _FoldNLL.apply(y, x, wf, bf, fp if params_grad else fp.detach(), stack, training, defer, gather)
    return stack.launch_fold_nll_forward(y, x, wf, bf, training, gather=gather)[2]


class _StackInverse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, h, stack: FusedStack, cond_index, training: bool):
        return stack.launch_inverse(z, h, cond_index, training)

    @staticmethod
    def backward(ctx, dy):
        raise NotImplementedError("bcnf_amd: CondRealNVP_v2.inverse is not differentiable (sampling path); "
                                  "run it under torch.no_grad().")


def _set_standalone_params(stack: FusedStack, flat, device):
    stack.flat = flat.detach().contiguous()
    if stack.qflat is None or stack.qflat.device != device:
        stack.qflat = torch.zeros(1, dtype=torch.float32, device=device)


def stack_forward(stack: FusedStack, y, h, training: bool, flat=None):
    y = y.contiguous()
    h = h.contiguous()
    if flat is not None:
        _set_standalone_params(stack, flat, y.device)
        fp = flat
        params_grad = flat.requires_grad
    else:
        stack.sync_grad_state()
        params_grad = stack.trainable[0].requires_grad
        fp = stack.flat_param
    if torch.is_grad_enabled():
        if params_grad or y.requires_grad or h.requires_grad:
            return _StackForward.apply(y, h, fp if params_grad else fp.detach(), stack, training)
    z, ldj, _, _ = stack.launch_forward(y, h, training, save=False)
    return z, ldj


def stack_inverse(stack: FusedStack, z, h, cond_index=None, training: bool = False, flat=None):
    z = z.contiguous()
    h = h.contiguous()
    if flat is not None:
        _set_standalone_params(stack, flat, z.device)
    if torch.is_grad_enabled() and (z.requires_grad or h.requires_grad):
        return _StackInverse.apply(z, h, stack, cond_index, training)
    return stack.launch_inverse(z, h, cond_index, training)

"""Host runtime of the wide-MLP coupling stack (trajectory_FC_large / trajectory_LSTM_large class).

Same contract as `FusedStack` (bcnf_amd/fused.py): one flat fp32 buffer of the trainable coupling parameters in
state_dict order with every nn.Parameter a view into it, the frozen orthonormal matrices in a second buffer, the
same autograd Functions (`_StackForward`, `_StackNLL`, `_StackInverse`) and the same launch_* methods, so
CondRealNVP_v2, TrainStep and the optimizer do not know which family runs. The arithmetic is in
libbcnf_amd.so (bcnf_amd/csrc/bcnf_wide.hip): fp32-MFMA GEMMs with fused bias/GELU/dropout/gradient epilogues
and per-sample link kernels; the condition projection h W0h^T of all blocks is one GEMM per pass.
"""
from __future__ import annotations

import ctypes
import math

import torch

from bcnf_amd import _native as N
from bcnf_amd.fused import FusedStack

_LOG2PI = math.log(2.0 * math.pi)


class WideStack(FusedStack):
    """Owns the flat parameter buffers of one wide-MLP coupling stack and drives the wide HIP kernels."""

    @property
    def supported(self) -> bool:
        return bool(N.lib().bcnf_wide_supported(self._pdesc))

    def counts(self):
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(N.lib().bcnf_wide_param_count(self._pdesc, ctypes.byref(a), ctypes.byref(b)), "bcnf_wide_param_count")
        return int(a.value), int(b.value)

    def _pack_into(self, out):
        N.check(N.lib().bcnf_wide_pack(self._pdesc, N.ptr(self.flat), N.ptr(self.qflat), N.ptr(out),
                                       N.stream_handle(self.flat.device)), "bcnf_wide_pack")

    def packed(self, fresh: bool = False):
        """Padded weight copies (bcnf_wide_pack). Re-packed on every call unless inside reuse_pack(); with
        fresh=True a private copy that a later forward cannot overwrite before this one's backward runs."""
        nbytes = N.query_i64(N.lib().bcnf_wide_packed_bytes, self._pdesc)
        if fresh and not self._pack_frozen:
            out = torch.empty(nbytes // 4, dtype=torch.float32, device=self.flat.device)
            self._pack_into(out)
            return out
        if self._packed is None:
            self._packed = torch.empty(nbytes // 4, dtype=torch.float32, device=self.flat.device)
        if not self._pack_frozen:
            self._pack_into(self._packed)
        return self._packed

    def workspace_bytes(self, batch: int, save: bool):
        return N.query_i64(N.lib().bcnf_wide_workspace_bytes, self._pdesc, ctypes.c_int64(batch),
                           ctypes.c_int32(int(save))), 0

    def _workspace(self, batch, save, dev):
        wb, _ = self.workspace_bytes(batch, save)
        return torch.empty(max(wb // 4, 1), dtype=torch.float32, device=dev)

    def _timed(self, name, fn):
        tm = self.timers
        if tm is None:
            return fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        tm.setdefault(name, []).append((e0, e1))
        return out

    # ------------------------------------------------------------------ launches
    def _forward(self, y, h, training, save, nll_part=None):
        self._check_inputs(y, h, "forward")
        if h.shape[0] != y.shape[0]:
            raise ValueError(f"bcnf_amd forward: {y.shape[0]} samples but {h.shape[0]} feature rows")
        B = y.shape[0]
        dev = y.device
        z = torch.empty_like(y)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        ws = self._workspace(B, save, dev)
        pk = self.packed(fresh=save)
        rc = self._timed("k_forward", lambda: N.lib().bcnf_wide_forward(
            self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(y), N.ptr(h), ctypes.c_int64(B), N.ptr(z), N.ptr(ldj),
            N.ptr(nll_part), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws), ctypes.c_int32(int(save)),
            N.stream_handle(dev)))
        N.check(rc, "bcnf_wide_forward")
        return z, ldj, rng, (ws, pk)

    def launch_forward(self, y, h, training: bool, save: bool, want_logp: bool = False):
        B = y.shape[0]
        part = torch.empty(B, dtype=torch.float32, device=y.device) if want_logp else None
        z, ldj, rng, saved = self._forward(y, h, training, save, part)
        if rng is not None:
            rng[1:2].add_(1)
        logp = None
        if want_logp:
            logp = -part - 0.5 * self.cfg.size * _LOG2PI
        return z, ldj, logp, saved

    def launch_backward(self, h, dz, dldj, training: bool, saved, want_dy: bool, want_dh: bool):
        return self._backward(h, None, dz, dldj, None, False, saved, want_dy, want_dh)

    def _backward(self, h, z, dz, dldj, dvals, nll, saved, want_dy, want_dh):
        ws, pk = saved
        B = h.shape[0]
        dev = h.device
        dparams = torch.empty_like(self.flat)
        dh = torch.empty_like(h) if want_dh else None
        dy = torch.empty((B, self.cfg.size), dtype=torch.float32, device=dev) if want_dy else None
        rc = self._timed("k_backward", lambda: N.lib().bcnf_wide_backward(
            self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(h), N.ptr(z), N.ptr(dz), N.ptr(dldj), N.ptr(dvals),
            ctypes.c_int32(int(nll)), ctypes.c_int64(B), N.ptr(ws), N.ptr(dy), N.ptr(dh), N.ptr(dparams),
            N.stream_handle(dev)))
        N.check(rc, "bcnf_wide_backward")
        return dy, dh, dparams

    def _finalize(self, ws, B, vals, training, save=True):
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        N.check(N.lib().bcnf_wide_nll_finalize(self._pdesc, N.ptr(ws), ctypes.c_int64(B), ctypes.c_int32(int(save)),
                                               N.ptr(vals), N.ptr(rng), N.ptr(self.guard),
                                               N.stream_handle(vals.device)), "bcnf_wide_nll_finalize")

    def launch_nll_forward(self, y, h, training: bool, finalize: bool = True):
        B = y.shape[0]
        if B == 0:
            raise ValueError("bcnf_amd: the NLL of an empty batch is undefined")
        z, ldj, _, saved = self._forward(y, h, training, True)
        vals = torch.empty(3, dtype=torch.float32, device=y.device)
        if finalize:
            self._finalize(saved[0], B, vals, training)
        return z, ldj, vals, saved

    def launch_nll_backward(self, h, z, dvals, training: bool, saved, want_dy: bool, want_dh: bool,
                            finalize_into=None):
        if finalize_into is not None:
            self._finalize(saved[0], h.shape[0], finalize_into, training)
        return self._backward(h, z, None, None, dvals, True, saved, want_dy, want_dh)

    # ------------------------------------------------------------------ folded last feature Linear
    # h = x Wf^T + bf enters the stack only through the condition projection: P = [x | 1] (W0h_all [Wf | bf])^T, and
    # the backward forms Gx = dZ0^T [x | 1] instead of dL/dh (include/bcnf_amd.h, bcnf_wide_fold_*).
    def fold_supported(self, in_features: int) -> bool:
        return in_features >= 1

    def _fold_operands(self, x, wf, bf, pk):
        B, X = x.shape
        xp = (X + 1 + 3) // 4 * 4
        dev = x.device
        x1 = torch.zeros((B, xp), dtype=torch.float32, device=dev)
        x1[:, :X] = x
        x1[:, X] = 1.0
        wfb = torch.zeros((wf.shape[0], xp), dtype=torch.float32, device=dev)
        wfb[:, :X] = wf
        if bf is not None:
            wfb[:, X] = bf
        rows = N.query_i64(N.lib().bcnf_wide_proj_rows, self._pdesc)
        wcb = torch.empty((rows, xp), dtype=torch.float32, device=dev)
        N.check(N.lib().bcnf_wide_fold_prepare(self._pdesc, N.ptr(pk), N.ptr(wfb), ctypes.c_int32(xp), N.ptr(wcb),
                                               N.stream_handle(dev)), "bcnf_wide_fold_prepare")
        return x1, wfb, wcb, xp

    def launch_fold_nll_forward(self, y, x, wf, bf, training: bool, finalize: bool = True):
        cfg = self.cfg
        if y.dim() != 2 or y.shape[1] != cfg.size:
            raise ValueError(f"bcnf_amd forward: expected (N, {cfg.size}) input, got {tuple(y.shape)}")
        if x.dim() != 2 or x.shape[0] != y.shape[0] or tuple(wf.shape) != (cfg.n_conditions, x.shape[1]):
            raise ValueError(f"bcnf_amd forward: folded features need x (N, X) and Wf ({cfg.n_conditions}, X), got "
                             f"{tuple(x.shape)} and {tuple(wf.shape)}")
        self._check_device(y, x, wf, bf)
        B = y.shape[0]
        if B == 0:
            raise ValueError("bcnf_amd: the NLL of an empty batch is undefined")
        dev = y.device
        z = torch.empty_like(y)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        drop = training and self.cfg.dropout > 0.0
        rng = self.rng_state() if drop else None
        ws = self._workspace(B, True, dev)
        pk = self.packed(fresh=True)
        x1, wfb, wcb, xp = self._fold_operands(x, wf, bf, pk)
        rc = self._timed("k_forward", lambda: N.lib().bcnf_wide_fold_forward(
            self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(y), N.ptr(x1), ctypes.c_int32(xp), N.ptr(wcb),
            ctypes.c_int64(B), N.ptr(z), N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
            N.stream_handle(dev)))
        N.check(rc, "bcnf_wide_fold_forward")
        vals = torch.empty(3, dtype=torch.float32, device=dev)
        if finalize:
            self._finalize(ws, B, vals, training)
        return z, ldj, vals, (ws, pk, x1, wfb, wcb, xp, x.shape[1])

    # Data parallel (TrainStep): (bucket, offset) -- the coupling gradients land in bucket[offset:offset + n], a view
    # that autograd adopts as .grad; and, with range_blocks (descending real-block ranges covering [0, nb)), the
    # backward runs range by range and calls on_range(lo, hi) with each finished range's bucket slice [lo, hi), so
    # the slice's all-reduce overlaps the rest of the backward (bcnf_wide_fold_backward_range).
    grad_bucket = None
    range_blocks = None
    on_range = None
    # TrainStep: with side_stream set, the coupling parameter gradients (bcnf_wide_fold_backward_phase 2) run on it
    # while the rest of the backward (the feature network's, fed by dL/dx from phase 1) continues on the launch
    # stream; join_side() makes the launch stream wait for them (before the gradients are read).
    side_stream = None
    _side_pending = None

    def join_side(self, param=None):
        """The launch stream waits for the side-stream parameter gradients of the last backward (no-op if none)."""
        pend, self._side_pending = self._side_pending, None
        if pend is None:
            return
        ev, stream, ptr, _keep = pend
        stream.wait_event(ev)
        if param is not None and param.requires_grad and (param.grad is None or param.grad.data_ptr() != ptr):
            # autograd copied the gradient (a clone on the launch stream) instead of adopting the side-stream buffer
            raise RuntimeError("bcnf_amd: the side-stream coupling gradient was not adopted as .grad")

    def block_offset(self, block: int) -> int:
        """Canonical flat offset of real block `block` (block = nb: the parameter count)."""
        return N.query_i64(N.lib().bcnf_wide_block_offset, self._pdesc, ctypes.c_int32(block))

    def launch_fold_nll_backward(self, z, dvals, training: bool, saved, want_x: bool, finalize_into=None):
        ws, pk, x1, wfb, wcb, xp, X = saved
        B = z.shape[0]
        dev = z.device
        if finalize_into is not None:
            self._finalize(ws, B, finalize_into, training)
        gx = torch.empty_like(wcb)
        off = None
        if self.grad_bucket is not None:
            bucket, off = self.grad_bucket
            dparams = bucket.narrow(0, off, self.flat.numel()).view_as(self.flat)
        else:
            dparams = torch.empty_like(self.flat)
        dwfb = torch.empty_like(wfb)
        dx = torch.empty((B, xp), dtype=torch.float32, device=dev) if want_x else None
        L = N.lib()
        stream = N.stream_handle(dev)
        args = (self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(x1), ctypes.c_int32(xp), N.ptr(wfb), N.ptr(wcb), N.ptr(z),
                N.ptr(dvals), ctypes.c_int64(B), N.ptr(ws), N.ptr(gx), N.ptr(dparams), N.ptr(dwfb), N.ptr(dx))
        if self.range_blocks and self.on_range is not None and off is not None:
            for lo, hi in self.range_blocks:
                N.check(L.bcnf_wide_fold_backward_range(*args, ctypes.c_int32(lo), ctypes.c_int32(hi), stream),
                        "bcnf_wide_fold_backward_range")
                self.on_range(off + self.block_offset(lo), off + self.block_offset(hi))
        elif self.side_stream is not None:
            if self._side_pending is not None:
                raise RuntimeError("bcnf_amd: a side-stream backward is still pending (join_side() not called)")
            cur = torch.cuda.current_stream(dev)
            rc = self._timed("k_backward", lambda: L.bcnf_wide_fold_backward_phase(*args, ctypes.c_int32(1), stream))
            N.check(rc, "bcnf_wide_fold_backward_phase")
            side = self.side_stream
            side.wait_stream(cur)
            N.check(L.bcnf_wide_fold_backward_phase(*args, ctypes.c_int32(2), ctypes.c_void_p(side.cuda_stream)),
                    "bcnf_wide_fold_backward_phase")
            ev = torch.cuda.Event()
            ev.record(side)
            # everything phase 2 reads stays alive until the join (freed afterwards on the launch stream, so a reuse
            # is ordered after the side stream's work); dparams itself must be adopted as .grad, not copied
            self._side_pending = (ev, cur, dparams.data_ptr(), (ws, pk, x1, wfb, wcb, z, dvals, gx, self.flat))
        else:
            rc = self._timed("k_backward", lambda: L.bcnf_wide_fold_backward(*args, stream))
            N.check(rc, "bcnf_wide_fold_backward")
        return dparams, dwfb[:, :X], dwfb[:, X], (dx[:, :X] if want_x else None)

    @torch.no_grad()
    def time_kernels(self, y, h, training: bool = True, iters: int = 20, fold=None):
        """Average device time (us) of the wide forward (save on) and backward launches, HIP events on the launch
        stream around `iters` back-to-back calls. fold = (x, Wf, bf): the folded training launches instead."""
        L = N.lib()
        dev = y.device
        stream = N.stream_handle(dev)
        B = y.shape[0]
        if fold is not None:
            z, _, vals, saved = self.launch_fold_nll_forward(y, *fold, training, finalize=False)
            ws, pk, x1, wfb, wcb, xp, _ = saved
            ldj = torch.empty(B, dtype=torch.float32, device=dev)
            gx = torch.empty_like(wcb)
            dparams = torch.empty_like(self.flat)
            dwfb = torch.empty_like(wfb)
            dx = torch.empty((B, xp), dtype=torch.float32, device=dev)
            rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
            calls = {
                "forward": lambda: L.bcnf_wide_fold_forward(
                    self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(y), N.ptr(x1), ctypes.c_int32(xp), N.ptr(wcb),
                    ctypes.c_int64(B), N.ptr(z), N.ptr(ldj), ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                    stream),
                "backward": lambda: L.bcnf_wide_fold_backward(
                    self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(x1), ctypes.c_int32(xp), N.ptr(wfb), N.ptr(wcb),
                    N.ptr(z), None, ctypes.c_int64(B), N.ptr(ws), N.ptr(gx), N.ptr(dparams), N.ptr(dwfb), N.ptr(dx),
                    stream),
            }
            return self._time_calls(calls, iters)
        z, _, vals, (ws, pk) = self.launch_nll_forward(y, h, training, finalize=False)
        ldj = torch.empty(B, dtype=torch.float32, device=dev)
        dparams = torch.empty_like(self.flat)
        dh = torch.empty_like(h)
        rng = self.rng_state() if (training and self.cfg.dropout > 0.0) else None
        calls = {
            "forward": lambda: L.bcnf_wide_forward(self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(y), N.ptr(h),
                                                   ctypes.c_int64(B), N.ptr(z), N.ptr(ldj), None,
                                                   ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(ws),
                                                   ctypes.c_int32(1), stream),
            "backward": lambda: L.bcnf_wide_backward(self._pdesc, N.ptr(self.flat), N.ptr(pk), N.ptr(h), N.ptr(z),
                                                     None, None, None, ctypes.c_int32(1), ctypes.c_int64(B),
                                                     N.ptr(ws), None, N.ptr(dh), N.ptr(dparams), stream),
        }
        return self._time_calls(calls, iters)

    @staticmethod
    def _time_calls(calls, iters):
        out = {}
        for name, fn in calls.items():
            N.check(fn(), name)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) * 1e3 / iters
        return out

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
        sb = N.query_i64(N.lib().bcnf_wide_inverse_scratch_bytes, self._pdesc, ctypes.c_int64(hr), ctypes.c_int64(n))
        scratch = torch.empty(max(sb // 4, 1), dtype=torch.float32, device=z.device)
        rc = N.lib().bcnf_wide_inverse(self._pdesc, N.ptr(self.flat), N.ptr(self.packed()), N.ptr(z), N.ptr(h),
                                       ctypes.c_int64(hr), N.ptr(cond_index), ctypes.c_int64(n), N.ptr(y),
                                       ctypes.c_int32(int(training)), N.ptr(rng), N.ptr(scratch),
                                       N.stream_handle(z.device))
        N.check(rc, "bcnf_wide_inverse")
        if drop:
            rng[1:2].add_(1)
        return y


class _WideFoldNLL(torch.autograd.Function):
    """vals = [loss, nll, mse] of the wide stack with the feature network's last Linear folded into the condition
    projection: inputs (y, x, Wf, bf, flat_param); gradients for x (the earlier feature layers), Wf, bf and flat_param."""

    @staticmethod
    def forward(ctx, y, x, wf, bf, flat_param, stack: WideStack, training: bool, defer: bool):
        z, _, vals, saved = stack.launch_fold_nll_forward(y, x, wf, bf, training, finalize=not defer)
        ctx.stack, ctx.training, ctx.saved, ctx.defer = stack, training, saved, defer
        ctx.has_bias = bf is not None
        ctx.save_for_backward(z, vals)
        return vals

    @staticmethod
    def backward(ctx, dvals):
        z, vals = ctx.saved_tensors
        need_x = ctx.needs_input_grad[1]
        dparams, dwf, dbf, dx = ctx.stack.launch_fold_nll_backward(
            z, dvals.contiguous(), ctx.training, ctx.saved, want_x=need_x, finalize_into=vals if ctx.defer else None)
        return (None, dx, dwf, (dbf if ctx.has_bias else None), (dparams if ctx.needs_input_grad[4] else None), None,
                None, None)


def stack_nll_wide_fold(stack: WideStack, y, x, wf, bf, training: bool, defer: bool = False):
    y = y.contiguous()
    x = x.contiguous()
    stack.sync_grad_state()
    fp = stack.flat_param if stack.trainable[0].requires_grad else stack.flat_param.detach()
    return _WideFoldNLL.apply(y, x, wf, bf, fp, stack, training, defer)


def make_stack(cfg, trainable, frozen, bind: bool = True) -> FusedStack:
    """The register-resident small family when the shape fits it (FC_small), else the wide-MLP family."""
    st = FusedStack(cfg, trainable, frozen, bind=False)
    if not st.supported:
        wd = WideStack(cfg, trainable, frozen, bind=False)
        if wd.supported:
            st = wd
    if bind:
        st.bind = True
        st.flatten()
    return st


__all__ = ["WideStack", "make_stack", "stack_nll_wide_fold"]

"""Optimizer step and gradient clipping of the bcnf Trainer on the library's HIP kernels.

The Trainer builds `torch.optim.Adam(model.parameters(), lr=...)` (src/bcnf/train/trainer.py:136) and,
after every `optimizer.step()`, calls `torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)`
(trainer.py:273-275). With the coupling stack held in one flat buffer (CondRealNVP_v2.flat_parameters())
torch's multi-tensor kernels see a handful of large tensors and parallelise poorly (one workgroup per
64 K-element chunk); `FusedAdam` runs the whole update as ONE launch over the concatenated index space
and emits the per-workgroup sums of squared gradients in the same pass, so the clip that follows is a
single further launch (`clip_grad_norm_after_step`).

Semantics are torch.optim.Adam's (amsgrad = maximize = False, optional L2 weight decay) with the step
count kept on the device (as Adam(capturable=True) does), so the step is HIP-graph capturable.
"""
from __future__ import annotations

import ctypes

import torch

from bcnf_amd import _native as N


def _groups(tensors, limit=N.MAX_TENSORS):
    for i in range(0, len(tensors), limit):
        yield tensors[i:i + limit]


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0:
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._partials = None      # per-workgroup sum(g^2) of the last step, consumed by the clip
        self._partials_for = None
        self._pending_steps = []   # step counts whose advance the following clip performs

    def _state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None, defer_step_count: bool = False, guard=None, bookkeep=None):
        """One Adam update. defer_step_count=True leaves the device step count to be advanced by the
        following clip_grad_norm_after_step (one launch less per training step). `guard` (device int32[4],
        include/bcnf_amd.h) turns the update into a no-op on a halted step. `bookkeep` = (cursor, log, counter)
        (clip_grad_norm_after_step's cursor / log, plus a zeroed device int32): the launch's last workgroup
        advances the step count and does that bookkeeping itself, for a step whose clip-after-step is
        unobservable (bcnf_adam_step_bookkeep); no clip may follow."""
        if bookkeep is not None:
            return self._step_bookkeep(guard, *bookkeep)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = N.lib()
        all_grads = []
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("bcnf_amd FusedAdam: parameters and grads must be contiguous fp32 GPU tensors")
            b1, b2 = group["betas"]
            dev = params[0].device
            for chunk in _groups(params):
                states = [self._state(p) for p in chunk]
                step = states[0]["step"]
                for st in states[1:]:                  # one shared device step per launch
                    if st["step"] is not step:
                        st["step"] = step
                grads = [p.grad for p in chunk]
                numel = N.i64_array([p.numel() for p in chunk])
                total = sum(p.numel() for p in chunk)
                part = torch.empty(int(L.bcnf_grad_partials(total)), dtype=torch.float32, device=dev)
                rc = L.bcnf_adam_step(len(chunk), N.ptr_array(chunk), N.ptr_array(grads),
                                      N.ptr_array([s["exp_avg"] for s in states]),
                                      N.ptr_array([s["exp_avg_sq"] for s in states]), numel, N.ptr(step),
                                      ctypes.c_double(group["lr"]), ctypes.c_double(b1), ctypes.c_double(b2),
                                      ctypes.c_double(group["eps"]), ctypes.c_double(group["weight_decay"]),
                                      N.ptr(part), ctypes.c_int32(0 if defer_step_count else 1), N.ptr(guard),
                                      N.stream_handle(dev))
                N.check(rc, "bcnf_adam_step")
                all_grads.append((chunk, grads, numel, part))
                if defer_step_count:
                    self._pending_steps.append(step)
        self._partials = all_grads
        self._partials_for = [p for chunk, _, _, _ in all_grads for p in chunk]
        return loss

    def can_bookkeep(self) -> bool:
        """Whether step(bookkeep=...) applies: one parameter group updated in one launch."""
        return len(self.param_groups) == 1 and 0 < len(self.param_groups[0]["params"]) <= N.MAX_TENSORS

    def _step_bookkeep(self, guard, cursor, log, counter):
        params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        if len(self.param_groups) != 1 or not params or len(params) > N.MAX_TENSORS:
            raise NotImplementedError("bcnf_amd FusedAdam: bookkeeping needs one group in one launch")
        group = self.param_groups[0]
        for p in params:
            if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                raise RuntimeError("bcnf_amd FusedAdam: parameters and grads must be contiguous fp32 GPU tensors")
        states = [self._state(p) for p in params]
        step = states[0]["step"]
        for st in states[1:]:
            if st["step"] is not step:
                st["step"] = step
        b1, b2 = group["betas"]
        cur, mod = cursor if cursor is not None else (None, 0)
        L = N.lib()
        rc = L.bcnf_adam_step_bookkeep(len(params), N.ptr_array(params), N.ptr_array([p.grad for p in params]),
                                       N.ptr_array([s["exp_avg"] for s in states]),
                                       N.ptr_array([s["exp_avg_sq"] for s in states]),
                                       N.i64_array([p.numel() for p in params]), N.ptr(step),
                                       ctypes.c_double(group["lr"]), ctypes.c_double(b1), ctypes.c_double(b2),
                                       ctypes.c_double(group["eps"]), ctypes.c_double(group["weight_decay"]),
                                       N.ptr(cur), ctypes.c_int64(mod), N.ptr(log[0] if log else None),
                                       N.ptr(log[1] if log else None), N.ptr(counter), N.ptr(guard),
                                       N.stream_handle(params[0].device))
        N.check(rc, "bcnf_adam_step_bookkeep")
        self._partials = None            # no clip may follow this step
        self._partials_for = None
        return None

    def fold_adam_spec(self, slots, cursor=None, log=None, counter=None, guard=None):
        """An N.BcnfFoldAdam for the folded backward tail (include/bcnf_amd.h): the update of exactly `slots` =
        (coupling flat parameter, feature weight, feature bias or None) -- all of this optimizer's parameters, one
        group -- fused where their gradients are produced, with step()'s bookkeep semantics. None if that does
        not describe this optimizer."""
        if len(self.param_groups) != 1:
            return None
        group = self.param_groups[0]
        live = [p for p in slots if p is not None]
        if {id(p) for p in live} != {id(p) for p in group["params"]} or len(live) != len(group["params"]):
            return None
        states = [self._state(p) for p in live]
        step = states[0]["step"]
        for st in states[1:]:
            if st["step"] is not step:
                st["step"] = step
        spec = N.BcnfFoldAdam()
        it = iter(states)
        for t, p in enumerate(slots):
            if p is None:
                continue
            st = next(it)
            spec.params[t] = p.data_ptr()
            spec.exp_avg[t] = st["exp_avg"].data_ptr()
            spec.exp_avg_sq[t] = st["exp_avg_sq"].data_ptr()
        b1, b2 = group["betas"]
        spec.step = step.data_ptr()
        spec.lr, spec.beta1, spec.beta2 = float(group["lr"]), float(b1), float(b2)
        spec.eps, spec.weight_decay = float(group["eps"]), float(group["weight_decay"])
        if cursor is not None:
            spec.advance_cursor, spec.cursor_modulo = cursor[0].data_ptr(), int(cursor[1])
        if log is not None:
            spec.log_values, spec.log_history = log[0].data_ptr(), log[1].data_ptr()
        spec.done_counter = counter.data_ptr()
        spec.guard = None if guard is None else guard.data_ptr()
        self._partials = None            # no clip may follow this step
        self._partials_for = None
        return spec

    @torch.no_grad()
    def clip_grad_norm_after_step(self, max_norm: float = 1.0, cursor=None, log=None, guard=None):
        """clip_grad_norm_(params, max_norm) for exactly the gradients the last step() consumed (unchanged
        since), reusing that step's squared-gradient partials. Also performs the end-of-step bookkeeping:
        a deferred step count, `cursor` = (device int64 counter, modulo) of an epoch walk, and
        `log` = (device values[3], history[n, 3] possibly pinned host memory): values -> history[cursor].
        `guard`: a halted step clips nothing and advances nothing. Returns the pre-clip total norm (device)."""
        if not self._partials:
            raise RuntimeError("bcnf_amd FusedAdam: clip_grad_norm_after_step() needs a preceding step()")
        L = N.lib()
        pending, self._pending_steps = self._pending_steps, []
        cur, mod = cursor if cursor is not None else (None, 0)
        if len(self._partials) != 1 or len(pending) > 1:   # several launches: generic path
            if log is not None or guard is not None:
                raise NotImplementedError("bcnf_amd FusedAdam: log/guard need a single-launch parameter set")
            norm = clip_grad_norm_(self._partials_for, max_norm)
            dev = norm.device
            for st in pending:
                N.check(L.bcnf_advance_counters(N.ptr(st), None, 0, N.stream_handle(dev)), "bcnf_advance_counters")
            if cur is not None:
                N.check(L.bcnf_advance_counters(None, N.ptr(cur), mod, N.stream_handle(dev)), "bcnf_advance_counters")
            return norm
        _, grads, numel, part = self._partials[0]
        dev = grads[0].device
        norm = torch.empty((), dtype=torch.float32, device=dev)
        rc = L.bcnf_clip_grad_norm(len(grads), N.ptr_array(grads), numel, N.ptr(part), ctypes.c_float(max_norm),
                                   N.ptr(norm), N.ptr(pending[0] if pending else None), N.ptr(cur),
                                   ctypes.c_int64(mod), N.ptr(log[0] if log else None), N.ptr(log[1] if log else None),
                                   N.ptr(guard), N.stream_handle(dev))
        N.check(rc, "bcnf_clip_grad_norm")
        return norm


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0):
    """torch.nn.utils.clip_grad_norm_ (2-norm) on the HIP kernels. Returns the total norm (device scalar)."""
    if norm_type != 2.0:
        raise NotImplementedError("bcnf_amd clip_grad_norm_: only the 2-norm (the Trainer's) is implemented")
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.zeros(())
    L = N.lib()
    dev = grads[0].device
    if len(grads) > N.MAX_TENSORS:
        # more tensors than one launch takes (a layerwise AnyGLU stack's per-layer parameters): the squared sums per
        # group on the HIP kernel, the total and the scaling as torch.nn.utils.clip_grad_norm_ does them
        sq = []
        for chunk in _groups(grads):
            numel = N.i64_array([g.numel() for g in chunk])
            part = torch.empty(int(L.bcnf_grad_partials(sum(g.numel() for g in chunk))), dtype=torch.float32,
                               device=dev)
            N.check(L.bcnf_grad_sumsq(len(chunk), N.ptr_array(chunk), numel, N.ptr(part), N.stream_handle(dev)),
                    "bcnf_grad_sumsq")
            sq.append(part[:-1].sum())              # the last slot is the clip's pre-reduce scratch
        norm = torch.stack(sq).sum().sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        torch._foreach_mul_(grads, coef)
        return norm
    numel = N.i64_array([g.numel() for g in grads])
    total = sum(g.numel() for g in grads)
    part = torch.empty(int(L.bcnf_grad_partials(total)), dtype=torch.float32, device=dev)
    stream = N.stream_handle(dev)
    N.check(L.bcnf_grad_sumsq(len(grads), N.ptr_array(grads), numel, N.ptr(part), stream), "bcnf_grad_sumsq")
    norm = torch.empty((), dtype=torch.float32, device=dev)
    N.check(L.bcnf_clip_grad_norm(len(grads), N.ptr_array(grads), numel, N.ptr(part), ctypes.c_float(max_norm),
                                  N.ptr(norm), None, None, ctypes.c_int64(0), None, None, None, stream),
            "bcnf_clip_grad_norm")
    return norm

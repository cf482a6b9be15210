"""Trainer-semantics training step on the fused kernels, with HIP-graph capture and data parallelism.

`TrainStep.step(y, traj)` performs exactly one `bcnf.train.Trainer._train_batch`
(src/bcnf/train/trainer.py:244-277):

    optimizer.zero_grad()
    z, h = model(y, *conditions, log_det_J=True, return_features=True)
    mse = MSE(prediction_head(h), y) if hybrid_weight > 0 else 0
    nll = inn_nll_loss(z, model.log_det_J)
    loss = (nll + mse * w) / (1 + w)
    loss.backward()
    [data parallel: every gradient packed into one bucket, ONE RCCL all-reduce (mean), grads = bucket views]
    optimizer.step()                                   # Adam
    clip_grad_norm_(parameters, max_norm=1.0)          # after the step, as the reference does
    loss.item(), nll.item(), mse.item()

MI355X specifics:
* hybrid_weight == 0 (every shipped config): forward + loss are ONE fused launch (`model.nll_loss`,
  bcnf_nll_forward) and loss.backward() is the fused NLL backward + deterministic slab reduce. A feature
  network that is one nn.Linear (trajectory_FC_small) is folded into the condition projection (no h, no
  dL/dh); other feature networks run on the library's MFMA GEMMs / PyTorch-ROCm.
* the coupling-stack parameters are ONE flat leaf (model.flat_parameters()); Adam is ONE launch over
  all parameters (bcnf_amd.optim.FusedAdam) that also emits the squared-gradient partials, so the
  clip after the step is one more launch.
* the whole step is captured once into a HIP graph and replayed (world > 1: the RCCL all-reduce runs
  between two captured segments). `step_indexed` also captures the batch gather from a
  device-resident pool (inside the folded path's pack launch), so a replay needs only the index copy.
* `run_epoch` replays 8 device-driven steps per graph. Only the last step of such a graph clips: the
  clip after the step (trainer.py:275) scales gradients the next step's backward overwrites and its norm
  is discarded, so every other step ("hidden") runs Adam with the bookkeeping instead -- on the folded
  path inside the backward tail itself (BcnfFoldAdam), with no Adam launch. run_epoch equals the per-step
  loop bit for bit (tests/test_gpu_train.py).
* the three logged values are stored by the clip launch straight into pinned host memory (a history
  row per batch of the epoch), so no copy node and, with `run_epoch`, no host sync per step: the epoch's
  steps are replayed back to back and the Trainer's per-batch divergence check (trainer.py:168) runs
  on the device (guard, include/bcnf_amd.h), halting the epoch in the state the reference raises in.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch
import torch.distributed as dist

from bcnf_amd.errors import TrainingDivergedError
from bcnf_amd.optim import FusedAdam, clip_grad_norm_
from bcnf_amd.utils import inn_nll_loss

GUARD_CHECK, GUARD_DIVERGED, GUARD_HALTED, GUARD_CHECK_GLOBAL, GUARD_WORDS = 0, 1, 2, 3, 4    # include/bcnf_amd.h


class TrainStep:
    def __init__(self, model, lr: float = 2e-4, hybrid_weight: float = 0.0, capture: bool = True,
                 max_norm: float = 1.0, process_group=None, overlap_ranges: int = 0):
        # An AnyGLU coupling stack (layer="AnyGLU", reference layers.py:9-31, dev configs) has no fused kernel family:
        # it runs layer by layer (its Linear layers on the library's MFMA GEMMs, autograd), so its step is the same
        # Trainer step run eagerly over model.parameters() -- FusedAdam, the clip after the step, the bucket
        # all-reduce -- without graph capture or the device divergence guard (the loss is checked on the host).
        self.layerwise = getattr(model, "_path", "fused") == "layerwise"
        self.model = model
        self.params = [p for p in model.parameters() if p.requires_grad] if self.layerwise \
            else model.flat_parameters()
        self.hybrid_weight = float(hybrid_weight)
        self.max_norm = max_norm
        self.capture = capture and not self.layerwise
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.opt = FusedAdam(self.params, lr=lr)
        self.mse = torch.nn.MSELoss()
        self.fused_loss = self.hybrid_weight == 0.0
        self._cot = None
        self._graphs = None
        self._static = None
        self._pool = None
        self._multi = {}        # steps -> (graph, steps, grads): run_epoch's multi-step graphs (world 1)
        self._single_grads = None
        self._rebind = False    # .grad currently points at buffers other than the single-step graph's
        self._book = None       # Adam's finished-workgroup counter (bcnf_adam_step_bookkeep)
        self._g2_hidden = None  # data parallel: update segment without the (unobservable) clip
        self._g21 = None        # data parallel: hidden update + the next step's forward/backward, one graph
        self._cond_shape = None  # (per-sample condition shape, its size) when the pool rows are padded
        self._epoch = None      # (order, cursor, n_batches, batch) for the device-cursor batch walk
        self._bucket = None     # data parallel: every gradient in one buffer, one all-reduce per step
        self._n_grad = 0        # gradient floats in the bucket; the 3 logged values follow (reduced with them)
        self._gvals = None      # data parallel: the all-reduced (loss, nll, mse) -- a view of the bucket tail
        self._packed_inplace = False   # the last bucket pack found the gradients already in place
        self._host_cursor = 0   # host mirror of the epoch cursor (the history row of the next step)
        # data parallel, wide family: the backward runs in `overlap_ranges` block ranges and each finished range's
        # bucket slice is all-reduced (async) while the rest of the backward runs; eager steps (the collectives are
        # issued between kernel launches, outside any captured graph), joined before the update
        self.overlap_ranges = 0
        self._works = []        # in-flight all-reduces of bucket slices, and the slices [lo, hi) they cover
        self._reduced = []
        self._hooks = None      # data parallel: the stack attributes _stack_hooks installs around each backward
        from bcnf_amd.wide import WideStack
        if self.world > 1 and overlap_ranges > 0 and isinstance(getattr(model, "fused", None), WideStack):
            self.overlap_ranges = min(int(overlap_ranges), model.fused.cfg.n_blocks)
            self.capture = False
        dev = self.params[0].device
        # wide family, ranges off, BCNF_WIDE_SIDE=1: the parameter-gradient phase of the folded backward overlaps the
        # feature network's backward on a side stream. Off by default: measured same-box it gains 0.3%
        # on FC_large and costs 5.6% on LSTM_large (the MIOpen RNN backward's serial kernels lose CUs to it)
        self._side = None
        if dev.type == "cuda" and self.overlap_ranges == 0 and isinstance(getattr(model, "fused", None), WideStack) \
                and os.environ.get("BCNF_WIDE_SIDE", "0") != "0":
            self._side = torch.cuda.Stream(device=dev)
        self._guard = None
        self._hist = None
        if dev.type == "cuda":
            self._guard = torch.zeros(GUARD_WORDS, dtype=torch.int32, device=dev)
            model.fused.guard = self._guard
            self._hist = torch.zeros((1, 3), dtype=torch.float32, pin_memory=True)

    # ------------------------------------------------------------------ step pieces
    def _forward_backward(self, y, traj, gather=None, adam=None):
        with self._stack_hooks(), self._side_overlap():
            return self._forward_backward_body(y, traj, gather, adam)

    @contextlib.contextmanager
    def _side_overlap(self):
        """Wide family: the coupling parameter gradients on a second stream, overlapping the feature network's
        backward (WideStack.side_stream); joined before anything reads the gradients (bucket pack, all-reduce, Adam).
        Eager or captured alike (the fork and join are stream-event edges of the graph)."""
        if self._side is None:
            yield
            return
        st = self.model.fused
        st.side_stream = self._side
        try:
            yield
        except BaseException:
            # the body raised (e.g. a divergence or launch error, possibly before autograd adopted the side buffer):
            # join the stream but skip the adoption check, so the original error is the one reported
            st.side_stream = None
            st.join_side(None)
            raise
        st.side_stream = None
        st.join_side(st.flat_param)

    def _forward_backward_body(self, y, traj, gather=None, adam=None):
        self.opt.zero_grad(set_to_none=True)
        if self.fused_loss:
            # reduced in the backward launch; a deferred gather runs inside the pack launch
            vals = self.model.nll_loss(y, traj, defer_reduction=True, gather=gather)
            if self._cot is None or self._cot.device != vals.device:
                self._cot = torch.tensor([1.0, 0.0, 0.0], device=vals.device)
            if adam is not None:                          # the optimizer step, inside the folded backward tail
                self.model.fused.pending_adam = adam(vals)
            torch.autograd.backward(vals, self._cot)      # loss.backward()
            if adam is not None and self.model.fused.pending_adam is not None:
                self.model.fused.pending_adam = None
                raise RuntimeError("bcnf_amd TrainStep: the folded backward did not take the fused Adam update")
            return vals.detach()
        z, h = self.model(y, traj, log_det_J=True, return_features=True)
        nll = inn_nll_loss(z, self.model.log_det_J)
        mse = self.mse(self.model.prediction_head(h), y)
        loss = (nll + mse * self.hybrid_weight) / (1 + self.hybrid_weight)
        loss.backward()
        return torch.stack([loss.detach(), nll.detach(), mse.detach()])

    def _pack_grads(self):
        """All gradients -> one contiguous bucket, so the data-parallel exchange is ONE collective per step whatever
        the number of feature-network tensors (FC_large: 17, LSTM_large: 19). Gradients the backward already wrote
        into their bucket slots (the folded backwards, FusedStack / WideStack.grad_bucket) are not copied."""
        grads = [p.grad for p in self.params]
        if any(g is None for g in grads):
            raise RuntimeError("bcnf_amd TrainStep: a parameter received no gradient")
        if self._bucket is None:
            self._alloc_bucket(grads[0].device)
        base, off, slots = self._bucket.data_ptr(), 0, []
        for g in grads:
            slots.append((g, off, g.is_contiguous() and g.data_ptr() == base + 4 * off))
            off += g.numel()
        self._packed_inplace = all(ok for _, _, ok in slots)
        if self._packed_inplace:
            return
        if not any(ok for _, _, ok in slots):
            torch.cat([g.reshape(-1) for g in grads], out=self._bucket[:self._n_grad])
            return
        for g, o, ok in slots:
            if ok:
                continue
            if any(lo < o + g.numel() and o < hi for lo, hi in self._reduced):
                raise RuntimeError("bcnf_amd TrainStep: a gradient of an already all-reduced bucket slice is not in "
                                   "its slot")
            self._bucket[o:o + g.numel()].copy_(g.reshape(-1))

    def _alloc_bucket(self, dev):
        """The gradient bucket + a 4-float tail holding the step's logged (loss, nll, mse): the one all-reduce of the
        step also averages them, so every rank logs -- and judges divergence on -- the global loss."""
        self._n_grad = sum(p.numel() for p in self.params)
        self._bucket = torch.zeros(self._n_grad + 4, dtype=torch.float32, device=dev)
        self._gvals = self._bucket[self._n_grad:self._n_grad + 3]

    def _setup_bucket(self):
        """Data parallel: allocate the gradient bucket up front and let the folded backwards write their gradients
        into it (no copy before the all-reduce): the small family's (coupling + feature Linear,
        FusedStack.grad_bucket), the wide family's coupling gradients (WideStack.grad_bucket), the latter range by
        range when overlap_ranges is set. The stack hooks are installed only around this step's own backward
        (_stack_hooks), so a backward outside the TrainStep never writes into the bucket or issues collectives."""
        if self.world == 1 or self._bucket is not None:
            return
        self._alloc_bucket(self.params[0].device)
        lin = self.model._fold_linear() if hasattr(self.model, "_fold_linear") else None
        if lin is None or not self.fused_loss or self.layerwise:
            return
        offs, off = {}, 0
        for p in self.params:
            offs[id(p)] = off
            off += p.numel()
        fp = self.model.fused.flat_param
        from bcnf_amd.wide import WideStack
        if isinstance(self.model.fused, WideStack):
            if id(fp) not in offs:
                return
            st = self.model.fused
            hooks = {"grad_bucket": (self._bucket, offs[id(fp)])}
            if self.overlap_ranges > 0:
                nb, r = st.cfg.n_blocks, self.overlap_ranges
                cuts = [round(nb * i / r) for i in range(r + 1)]
                hooks["range_blocks"] = [(cuts[i - 1], cuts[i]) for i in range(r, 0, -1) if cuts[i] > cuts[i - 1]]
                hooks["on_range"] = self._reduce_range
            self._hooks = hooks
            return
        if len(self.params) != (3 if lin.bias is not None else 2) or id(fp) not in offs or id(lin.weight) not in offs:
            return
        self._hooks = {"grad_bucket": (self._bucket, (offs[id(fp)], offs[id(lin.weight)],
                                                      offs[id(lin.bias)] if lin.bias is not None else 0))}

    @contextlib.contextmanager
    def _stack_hooks(self):
        """The bucket / range hooks on the fused stack for the duration of this step's forward + backward (eager or
        being captured), removed afterwards even when the step raises."""
        st = self.model.fused
        if not self._hooks:
            yield
            return
        for k, v in self._hooks.items():
            setattr(st, k, v)
        try:
            yield
        finally:
            for k in self._hooks:
                setattr(st, k, None)

    def _drain_slices(self):
        """Join and forget slice all-reduces a previous step left in flight (it raised between issuing them and the
        update's join), so this step neither skips those slices nor waits on stale handles."""
        works, self._works = self._works, []
        self._reduced.clear()
        for w in works:
            try:
                w.wait()
            except Exception:       # the failed step's own error was already raised to the caller
                pass

    def _bind_grads(self):
        """Every .grad becomes a view of the (reduced) bucket: Adam and the clip read it in place."""
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self._bucket[off:off + n].view_as(p)
            off += n

    def _reduce_bucket(self):
        """Sum over ranks of the gradient bucket: ONE RCCL all-reduce per step (the 1/world scaling runs inside
        the captured update segment, _scale_bucket). With slices already in flight (overlap_ranges), the rest of the
        bucket -- the feature-network gradients and the logged values -- then a join on every slice."""
        if not self._works:
            dist.all_reduce(self._bucket, op=dist.ReduceOp.SUM, group=self.pg)
            return
        lo = 0
        for a, b in sorted(self._reduced) + [(self._bucket.numel(), self._bucket.numel())]:
            if a > lo:
                dist.all_reduce(self._bucket[lo:a], op=dist.ReduceOp.SUM, group=self.pg)
            lo = max(lo, b)
        for w in self._works:
            w.wait()
        self._works.clear()
        self._reduced.clear()

    def _reduce_range(self, lo: int, hi: int):
        """A finished block range's bucket slice [lo, hi): its all-reduce runs while the backward continues
        (WideStack.on_range); the update joins it (_reduce_bucket)."""
        self._works.append(dist.all_reduce(self._bucket[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
        self._reduced.append((lo, hi))

    def _scale_bucket(self):
        self._bucket.mul_(1.0 / self.world)

    def _allreduce(self, vals=None):
        """Eager data-parallel exchange; returns the all-reduced logged values (or `vals` at world 1)."""
        if self.world == 1:
            return vals
        self._pack_grads()
        if vals is not None:
            self._gvals.copy_(vals)
        self._reduce_bucket()
        self._scale_bucket()
        self._bind_grads()
        return self._gvals if vals is not None else None

    def _check_global(self):
        """Data parallel: the divergence guard judged on the all-reduced loss (bcnf_guard_check_global)."""
        if self.world == 1 or self._guard is None:
            return
        from bcnf_amd import _native as N
        N.check(N.lib().bcnf_guard_check_global(N.ptr(self._gvals), N.ptr(self._guard),
                                                N.stream_handle(self._gvals.device)), "bcnf_guard_check_global")

    def _update(self, vals=None, clip: bool = True, epoch_book: bool = True):
        """Adam, then clip_grad_norm_ after the step (trainer.py:273-275); the clip launch also advances the
        Adam step count and, in epoch mode, the batch cursor, and stores the logged values into the pinned
        history (end-of-step bookkeeping, no extra launch). epoch_book=False: a batch from outside the epoch
        order (step_indexed while an order is set) -- no cursor advance and no history row."""
        if self.world > 1 and vals is not None:
            vals = self._gvals              # every rank logs the global values and halts on the same step
            self._check_global()
        cursor = (self._epoch[1], self._epoch[2]) if (self._epoch is not None and epoch_book) else None
        log = (vals, self._hist) if (vals is not None and self._hist is not None and epoch_book) else None
        if not clip:
            # a step inside a multi-step graph that the next step's backward follows: its clip-after-step
            # would only scale gradients that are overwritten before anyone can read them (the reference
            # discards the norm), so Adam's last workgroup does the step's bookkeeping and no clip runs
            if self._book is None:
                self._book = torch.zeros(1, dtype=torch.int32, device=self.params[0].device)
            self.opt.step(guard=self._guard, bookkeep=(cursor, log, self._book))
            return
        if self.layerwise:
            # eager only: the values go back to the caller directly (no history row); no device guard, and the
            # parameter list may span several Adam launches (the generic clip of FusedAdam)
            self.opt.step(defer_step_count=True)
            self.opt.clip_grad_norm_after_step(self.max_norm, cursor=cursor)
            return
        self.opt.step(defer_step_count=True, guard=self._guard)
        self.opt.clip_grad_norm_after_step(self.max_norm, cursor=cursor, log=log, guard=self._guard)

    def broadcast_parameters(self, src: int = 0):
        """Identical initial replicas (the RNG-seeded init differs per process otherwise)."""
        if self.world == 1:
            return
        with torch.no_grad():
            frozen = [] if self.layerwise else [self.model.fused.qflat]   # layerwise: Q are model parameters
            for p in list(self.model.parameters()) + frozen:
                dist.broadcast(p.data, src=src, group=self.pg)

    # ------------------------------------------------------------------ eager / graph
    def eager_step(self, y, traj, gather=None, epoch_book: bool = True):
        self._drain_slices()
        self._setup_bucket()
        vals = self._forward_backward(y, traj, gather)
        vals = self._allreduce(vals)
        self._update(vals, epoch_book=epoch_book)
        self._rebind = self._graphs is not None     # .grad now holds this step's buffers, not a graph's
        # world > 1: vals is a view of the bucket tail, which the next step overwrites
        return vals.clone() if self.world > 1 else vals

    def _gather(self, defer: bool = False):
        """Pool rows of the current batch, both tensors in one native launch: the static index buffer, or
        (epoch mode) batch `cursor` of the device-resident epoch order, the cursor advancing on the device.
        defer=True returns (y, traj, spec): when the step takes the folded path, spec is the gather (not yet
        launched) for the pack launch to run (bcnf_pack_params_fold), else None and the gather has run."""
        from bcnf_amd import _native as N
        py, pt = self._pool
        n = self._epoch[3] if self._epoch is not None else self._static[2].shape[0]
        y = torch.empty((n,) + tuple(py.shape[1:]), dtype=py.dtype, device=py.device)
        t = torch.empty((n,) + tuple(pt.shape[1:]), dtype=pt.dtype, device=pt.device)
        cy = py[0].numel()
        ct = pt[0].numel()
        if defer and self.fused_loss and self.fuse_gather and not self.layerwise and \
                self.model._foldable_linear(y, (self._unpad(t),)) is not None:
            epoch = self._epoch is not None
            spec = N.BcnfGather2(idx=(self._epoch[0] if epoch else self._static[2]).data_ptr(),
                                 cursor=self._epoch[1].data_ptr() if epoch else None, n=n,
                                 src0=py.data_ptr(), cols0=cy, dst0=y.data_ptr(),
                                 src1=pt.data_ptr(), cols1=ct, dst1=t.data_ptr())
            return y, self._unpad(t), spec
        st = N.stream_handle(py.device)
        if self._epoch is not None:
            order, cursor = self._epoch[0], self._epoch[1]
            N.check(N.lib().bcnf_gather_batch(N.ptr(order), N.ptr(cursor), n, N.ptr(py), cy, N.ptr(y), N.ptr(pt), ct,
                                              N.ptr(t), st), "bcnf_gather_batch")
        else:
            N.check(N.lib().bcnf_gather_rows2(N.ptr(self._static[2]), n, N.ptr(py), cy, N.ptr(y), N.ptr(pt), ct,
                                              N.ptr(t), st), "bcnf_gather_rows2")
        if defer:
            return y, self._unpad(t), None
        return y, self._unpad(t)

    def _unpad(self, t):
        """A batch of the padded condition pool as the (n, *cond_shape) view the model expects (row stride = the
        padded width; the folded path reads it in place with float4 loads)."""
        if self._cond_shape is None:
            return t
        shape, X = self._cond_shape
        return t[:, :X].view((t.shape[0],) + shape)

    def _pool_rows(self, idx):
        py, pt = self._pool
        return py.index_select(0, idx), self._unpad(pt.index_select(0, idx))

    def _snapshot(self):
        with torch.no_grad():
            params = [p.detach().clone() for p in self.model.parameters()]
            opt = {id(p): {k: v.clone() for k, v in st.items() if torch.is_tensor(v)}
                   for p, st in self.opt.state.items()}
            rng = self.model.fused.rng_state().clone()
            cur = self._epoch[1].clone() if self._epoch is not None else None
        return params, opt, rng, cur

    def _restore(self, snap):
        params, opt, rng, cur = snap
        with torch.no_grad():
            if cur is not None:
                self._epoch[1].copy_(cur)
            for p, v in zip(self.model.parameters(), params):
                p.copy_(v)
            for p, st in self.opt.state.items():
                saved = opt.get(id(p))
                for k, v in st.items():
                    if torch.is_tensor(v):
                        v.copy_(saved[k]) if saved is not None else v.zero_()
            self.model.fused.rng_state().copy_(rng)

    def _build_graphs(self, y, traj, idx=None, warmup: int = 2):
        """Warm up (allocations, kernel attributes) on a side stream, undo the warm-up's updates, then
        capture: the first step() applies exactly one update, like every later one."""
        self._setup_bucket()
        self._static = (y.clone(), traj.clone(), None if idx is None else idx.clone())
        sy, st, _ = self._static
        indexed = idx is not None
        snap = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                if indexed:
                    self.eager_step(*self._gather(defer=True))
                else:
                    self.eager_step(sy, st)
            self._restore(snap)
        torch.cuda.current_stream().wait_stream(s)
        self.opt.zero_grad(set_to_none=True)
        # the three logged values are stored into the pinned history by the clip launch: the host reads
        # them after a stream sync, without a device-to-host copy node
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            spec = None
            if indexed:
                sy, st, spec = self._gather(defer=True)
            vals = self._forward_backward(sy, st, spec)
            if self.world == 1:
                self._update(vals)
            else:
                self._pack_grads()          # the bucket copy is part of the captured step
                self._gvals.copy_(vals)     # the logged values travel with the gradients
        g2 = None
        if self.world > 1:
            self._bind_grads()              # the update reads the reduced bucket
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._scale_bucket()
                self._update(vals)
            # the update segment of a step whose clip-after-step is unobservable (every run_epoch step but the
            # last: the next step's backward overwrites the gradients): Adam with the bookkeeping, no clip launch
            if self.skip_hidden_clips and self.opt.can_bookkeep():
                if self._book is None:
                    self._book = torch.zeros(1, dtype=torch.int32, device=self.params[0].device)
                self._g2_hidden = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g2_hidden):
                    self._scale_bucket()
                    self._update(vals, clip=False)
                if indexed:
                    # step i's hidden update and step i+1's gather / forward / backward / bucket in ONE graph: one
                    # inter-graph idle per step instead of two (run_epoch); step i+1's logged values are copied
                    # into g1's buffer, which every update segment logs from
                    self._g21 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self._g21):
                        self._scale_bucket()
                        self._update(vals, clip=False)
                        sy2, st2, spec2 = self._gather(defer=True)
                        vals2 = self._forward_backward(sy2, st2, spec2)
                        self._pack_grads()
                        self._gvals.copy_(vals2)
                        vals.copy_(vals2)
                    self._bind_grads()
        self._graphs = (g1, g2, vals)
        self._single_grads = [p.grad for p in self.params]   # what .grad shows after a g1 replay

    def step(self, y, traj):
        """One training step; returns (loss, nll, mse) as Python floats (the Trainer's three .item())."""
        vals = self.step_async(y, traj)
        if not self.capture:
            return tuple(vals.tolist())
        return self._host_values()

    def _host_values(self, row: int = 0):
        """The step's three logged values (the Trainer's .item() calls): one stream sync, then a read of the
        pinned history row the clip launch stored them in."""
        torch.cuda.current_stream().synchronize()
        return tuple(self._hist[row].tolist())

    def step_async(self, y, traj):
        if not self.capture:
            return self.eager_step(y, traj)
        if self._graphs is None:
            self._build_graphs(y, traj)
        sy, st, _ = self._static
        if sy is None or y.shape != sy.shape or traj.shape != st.shape:
            # a batch of another size (the DataLoader's last, drop_last=False): the captured graph holds buffers of
            # the first batch's size, so this one runs eagerly on the same kernels and optimizer state
            return self.eager_step(y, traj)
        sy.copy_(y, non_blocking=True)
        st.copy_(traj, non_blocking=True)
        return self._replay()

    # ------------------------------------------------------------------ device-resident data pool
    def set_pool(self, y_pool, traj_pool):
        """Serve batches by index from device-resident tensors (the gather becomes part of the graph)."""
        if self._graphs is not None:
            raise RuntimeError("set_pool() must precede the first step")
        for t in (y_pool, traj_pool):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise ValueError("set_pool: contiguous fp32 device tensors required")
        # the folded feature Linear (cnf.py fold_pool_width) reads x rows with float4 loads when they are 16-byte
        # aligned: zero-pad the pool's rows (90 -> 92 floats for FC_small) once, here
        self._cond_shape = None
        w = self.model.fold_pool_width(traj_pool) if hasattr(self.model, "fold_pool_width") else None
        if w is not None:
            X = traj_pool[0].numel()
            padded = torch.zeros((traj_pool.shape[0], w), dtype=traj_pool.dtype, device=traj_pool.device)
            padded[:, :X] = traj_pool.reshape(traj_pool.shape[0], X)
            self._cond_shape = (tuple(traj_pool.shape[1:]), X)
            traj_pool = padded
        self._pool = (y_pool, traj_pool)

    def step_indexed(self, idx):
        """step(pool_y[idx], pool_traj[idx]) with the gather captured in the graph."""
        if self._pool is None:
            raise RuntimeError("step_indexed() needs set_pool()")
        self._check_indices(idx)
        idx = idx.to(device=self._pool[0].device, dtype=torch.int64).contiguous()
        if self._epoch is not None:
            # a batch outside the epoch order (the ragged remainder of an epoch, drop_last=False): the epoch graphs
            # walk the device cursor and write history rows, so this one runs eagerly on the same kernels and
            # optimizer state without touching the cursor or the history
            return tuple(self.eager_step(*self._pool_rows(idx), epoch_book=False).tolist())
        if not self.capture:
            self._static = (None, None, idx)
            return tuple(self.eager_step(*self._gather()).tolist())
        if self._graphs is None:
            self._build_graphs(*self._pool_rows(idx), idx=idx)
        if self._static[2] is None or idx.shape != self._static[2].shape:
            return tuple(self.eager_step(*self._pool_rows(idx)).tolist())     # another batch size: eager
        self._static[2].copy_(idx, non_blocking=True)
        self._replay()
        return self._host_values()

    def _check_indices(self, idx):
        """Pool indices in range (the reference's DataLoader raises IndexError; the device gather would read out of
        bounds), before anything is launched. Host indices (a DataLoader's) are checked on the host, no device sync;
        device-resident indices cost one host round trip."""
        if idx.numel() == 0:
            return
        lo, hi = torch.aminmax(idx if idx.device.type == "cpu" else idx.to(torch.int64))
        n = self._pool[0].shape[0]
        if int(lo) < 0 or int(hi) >= n:
            raise IndexError(f"bcnf_amd TrainStep: batch index out of range [0, {n}) (got {int(lo)}..{int(hi)})")

    # ------------------------------------------------------------------ device-resident epoch order
    def set_epoch(self, order, batch: int):
        """Walk `order` (device int64, n_batches * batch pool indices, e.g. concatenated shuffled epochs)
        batch by batch with step_epoch(); the graph reads batch `cursor` and advances the cursor itself, so
        a step needs no host-to-device traffic. A later call replaces the order (same size) and rewinds."""
        if self._pool is None:
            raise RuntimeError("set_epoch() needs set_pool()")
        order = order.to(dtype=torch.int64).contiguous()
        nb = order.numel() // batch
        if nb < 1 or order.numel() != nb * batch:
            # whole batches only: a ragged last batch (drop_last=False) goes through step_indexed, which runs a
            # batch of another size eagerly
            raise ValueError(f"set_epoch: order must hold a whole number of batches ({order.numel()} indices, "
                             f"batch {batch}); pass the remainder to step_indexed()")
        self._check_indices(order)
        if self._epoch is None:
            if self._graphs is not None:
                raise RuntimeError("set_epoch() must precede the first step of a non-epoch TrainStep")
            dev = order.device
            self._epoch = (order.clone(), torch.zeros(1, dtype=torch.int64, device=dev), nb, batch)
            self._hist = torch.zeros((nb, 3), dtype=torch.float32, pin_memory=True)
        else:
            o, cursor, nb0, b0 = self._epoch
            if nb != nb0 or batch != b0:
                raise ValueError("set_epoch: a captured TrainStep keeps its order size")
            o.copy_(order)
            cursor.zero_()
        self._host_cursor = 0

    def step_epoch(self):
        """The next batch of the epoch order (see set_epoch)."""
        if self._epoch is None:
            raise RuntimeError("step_epoch() needs set_epoch()")
        row = self._host_cursor
        self._host_cursor = (row + 1) % self._epoch[2]
        if not self.capture:
            return tuple(self.eager_step(*self._gather()).tolist())
        self._ensure_epoch_graphs()
        self._replay()
        return self._host_values(row)

    def _ensure_epoch_graphs(self):
        if self._graphs is None:
            y, t = self._gather()
            self._build_graphs(y, t, idx=torch.zeros(1, dtype=torch.int64, device=y.device))

    def run_epoch(self, n_steps=None, check_divergence: bool = False):
        """The remaining batches of the epoch order (or the next n_steps of them) replayed back to back with
        ONE host sync at the end; returns their (loss, nll, mse) triples in order -- the values the
        Trainer's per-batch .item() calls read (trainer.py:166-173). With check_divergence (the Trainer
        checks after epoch 10) a loss > 1e5 or NaN halts the epoch on the device right after that step's
        update and TrainingDivergedError is raised here, with the model, optimizer, RNG offset and cursor
        as the reference leaves them when it raises (only .grad holds the discarded next batch's gradient)."""
        if self._epoch is None:
            raise RuntimeError("run_epoch() needs set_epoch()")
        nb = self._epoch[2]
        start = self._host_cursor
        n = nb - start if n_steps is None else int(n_steps)
        if n < 0 or start + n > nb:
            raise ValueError(f"run_epoch: {n} steps from batch {start} exceed the epoch's {nb} batches")
        if n == 0:
            return []
        if not self.capture or not self.fused_loss:    # per-step host check (the device guard sits in
            out = []                                     # the fused loss finalize), right after each update
            for i in range(n):                           # as trainer.py:166-168 does
                v = self.step_epoch()
                out.append(v)
                if check_divergence and (v[0] > 1e5 or math.isnan(v[0])):
                    raise TrainingDivergedError(f"Loss exploded to {v[0]} at batch {start + i}")
            return out
        self._ensure_epoch_graphs()
        self._guard.zero_()
        if check_divergence:        # data parallel: judged on the all-reduced loss, the same on every rank
            self._guard[GUARD_CHECK if self.world == 1 else GUARD_CHECK_GLOBAL] = 1
        i = 0
        if self.world == 1 and self.epoch_unroll > 1:
            for k in self._unroll_sizes():
                if n - i < k:
                    continue
                g, _, grads = self._multi_graph(k)
                while n - i >= k:
                    g.replay()
                    i += k
                self._bind(grads)
                self._rebind = True
        if self.world > 1 and self._g21 is not None and n >= 2:
            g1, g2, _ = self._graphs          # g1, then (all-reduce, g21) per later step, then the last update
            g1.replay()
            for _ in range(n - 1):
                self._reduce_bucket()
                self._g21.replay()
            self._reduce_bucket()
            g2.replay()
            i = n
        while i < n:
            self._replay(hidden=i < n - 1)
            i += 1
        torch.cuda.current_stream().synchronize()
        vals = [tuple(r) for r in self._hist[start:start + n].tolist()]
        self._host_cursor = (start + n) % nb
        if check_divergence and int(self._guard[GUARD_DIVERGED].item()):
            for i, v in enumerate(vals):
                if v[0] > 1e5 or math.isnan(v[0]):
                    self._host_cursor = (start + i + 1) % nb
                    self._guard.zero_()
                    raise TrainingDivergedError(f"Loss exploded to {v[0]} at batch {start + i}")
        return vals

    # Steps per captured graph in run_epoch: a graph boundary costs ~9 us of idle GPU between two replays
    # (measured, r01j), so run_epoch replays `epoch_unroll` device-driven steps (cursor, RNG offset, Adam step,
    # history row all advance on the device) per launch and the remainder in graphs of epoch_unroll / 2, / 4, ...
    # steps (20 steps: 8 + 8 + 4, three launches instead of six) and a last single step.
    epoch_unroll = 8

    def _unroll_sizes(self):
        k, out = self.epoch_unroll, []
        while k > 1:
            out.append(k)
            k //= 2
        return out
    # The captured step runs the batch gather inside the folded path's pack launch (one launch fewer).
    fuse_gather = True
    # Inside a multi-step graph only the last step's clip-after-step is observable (see _update).
    skip_hidden_clips = True

    def _multi_graph(self, k: int):
        if k not in self._multi:
            self._bind(self._single_grads)         # every multi-step graph is captured from the same .grad state
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                slots = self._fold_adam_slots()
                for i in range(k):
                    hidden = i < k - 1 and self.skip_hidden_clips
                    sy, st, spec = self._gather(defer=True)
                    if hidden and slots is not None and self.model._foldable_linear(sy, (st,)) is not None:
                        # Adam of this step runs inside its folded backward tail (bcnf_fold_backward_tail)
                        self._forward_backward(sy, st, spec, adam=lambda v: self._fold_adam(slots, v))
                        continue
                    vals = self._forward_backward(sy, st, spec)
                    self._update(vals, clip=not (hidden and self.opt.can_bookkeep()))
            self._multi[k] = (g, k, [p.grad for p in self.params])
            self._bind(self._single_grads)
            self._rebind = False
        return self._multi[k]

    # Hidden steps of a folded model update their parameters inside the backward tail (no Adam launch).
    fuse_adam = True

    def _fold_adam_slots(self):
        """(coupling flat parameter, feature weight, feature bias) when the fused-Adam tail applies: the model
        folds its feature Linear and those are exactly this optimizer's parameters; else None."""
        if not self.fuse_adam or self.world != 1 or not self.fused_loss:
            return None
        lin = self.model._fold_linear() if hasattr(self.model, "_fold_linear") else None
        if lin is None:
            return None
        slots = (self.model.fused.flat_param, lin.weight, lin.bias)
        live = [p for p in slots if p is not None]
        if [id(p) for p in sorted(live, key=id)] != [id(p) for p in sorted(self.params, key=id)]:
            return None
        return slots

    def _fold_adam(self, slots, vals):
        if self._book is None:
            self._book = torch.zeros(1, dtype=torch.int32, device=self.params[0].device)
        cursor = (self._epoch[1], self._epoch[2]) if self._epoch is not None else None
        log = (vals, self._hist) if self._hist is not None else None
        spec = self.opt.fold_adam_spec(slots, cursor=cursor, log=log, counter=self._book, guard=self._guard)
        if spec is None:
            raise RuntimeError("bcnf_amd TrainStep: the optimizer does not match the fused-Adam slots")
        return spec

    def _bind(self, grads):
        """.grad = the gradient buffers of the graph that ran last (each captured graph owns its own)."""
        if grads is None:
            return
        for p, gr in zip(self.params, grads):
            p.grad = gr

    def prepare_epoch(self, n_steps: int):
        """Capture, without running anything, every graph a later run_epoch(n_steps) replays (the step graphs and,
        at world 1, the multi-step graph), so no capture lands inside a timed region."""
        if self._epoch is None or not self.capture or not self.fused_loss:
            return
        self._ensure_epoch_graphs()
        if self.world == 1 and self.epoch_unroll > 1:
            i = 0
            for k in self._unroll_sizes():
                if n_steps - i >= k:
                    self._multi_graph(k)
                    i += k * ((n_steps - i) // k)

    def _replay(self, hidden: bool = False):
        if self._rebind:
            self._bind(self._single_grads)
            self._rebind = False
        g1, g2, vals = self._graphs
        g1.replay()
        if g2 is not None:
            self._reduce_bucket()           # the one collective of the step, between the two graph segments
            (self._g2_hidden if hidden and self._g2_hidden is not None else g2).replay()
        return vals


__all__ = ["TrainStep", "FusedAdam", "clip_grad_norm_", "TrainingDivergedError"]

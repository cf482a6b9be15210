"""Trainer-semantics training step on the fused kernels, with HIP-graph capture and data parallelism.

`TrainStep.step(y, traj)` performs exactly one `bcnf.train.Trainer._train_batch`
(src/bcnf/train/trainer.py:244-277):

    optimizer.zero_grad()
    z, h = model(y, *conditions, log_det_J=True, return_features=True)
    mse = MSE(prediction_head(h), y) if hybrid_weight > 0 else 0
    nll = inn_nll_loss(z, model.log_det_J)
    loss = (nll + mse * w) / (1 + w)
    loss.backward()
    [data parallel: RCCL all-reduce (sum / world) of every gradient]
    optimizer.step()                                   # Adam
    clip_grad_norm_(parameters, max_norm=1.0)          # after the step, as the reference does
    loss.item(), nll.item(), mse.item()

MI355X specifics:
* hybrid_weight == 0 (every shipped config): forward + loss are ONE fused launch (`model.nll_loss`,
  bcnf_nll_forward) and loss.backward() is the fused NLL backward + deterministic slab reduce; the
  feature network's nn.Linear runs on the library's MFMA GEMMs. No elementwise loss kernels.
* the coupling-stack parameters are ONE flat leaf (model.flat_parameters()); Adam is ONE launch over
  all parameters (bcnf_amd.optim.FusedAdam) that also emits the squared-gradient partials, so the
  clip after the step is one more launch.
* the whole step is captured once into a HIP graph and replayed (world > 1: the RCCL all-reduce runs
  between two captured segments). `step_indexed` also captures the batch gather from a
  device-resident pool, so a replay needs only the index copy.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from bcnf_amd.optim import FusedAdam, clip_grad_norm_
from bcnf_amd.utils import inn_nll_loss


class TrainStep:
    def __init__(self, model, lr: float = 2e-4, hybrid_weight: float = 0.0, capture: bool = True,
                 max_norm: float = 1.0, process_group=None):
        self.model = model
        self.params = model.flat_parameters()
        self.hybrid_weight = float(hybrid_weight)
        self.max_norm = max_norm
        self.capture = capture
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        self.opt = FusedAdam(self.params, lr=lr)
        self.mse = torch.nn.MSELoss()
        self.fused_loss = self.hybrid_weight == 0.0
        self._cot = None
        self._graphs = None
        self._static = None
        self._pool = None

    # ------------------------------------------------------------------ step pieces
    def _forward_backward(self, y, traj):
        self.opt.zero_grad(set_to_none=True)
        if self.fused_loss:
            vals = self.model.nll_loss(y, traj)
            if self._cot is None or self._cot.device != vals.device:
                self._cot = torch.tensor([1.0, 0.0, 0.0], device=vals.device)
            torch.autograd.backward(vals, self._cot)      # loss.backward()
            return vals.detach()
        z, h = self.model(y, traj, log_det_J=True, return_features=True)
        nll = inn_nll_loss(z, self.model.log_det_J)
        mse = self.mse(self.model.prediction_head(h), y)
        loss = (nll + mse * self.hybrid_weight) / (1 + self.hybrid_weight)
        loss.backward()
        return torch.stack([loss.detach(), nll.detach(), mse.detach()])

    def _allreduce(self):
        if self.world == 1:
            return
        for p in self.params:
            if p.grad is not None:
                dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.pg)
                p.grad.mul_(1.0 / self.world)

    def _update(self):
        self.opt.step()
        self.opt.clip_grad_norm_after_step(self.max_norm)

    def broadcast_parameters(self, src: int = 0):
        """Identical initial replicas (the RNG-seeded init differs per process otherwise)."""
        if self.world == 1:
            return
        with torch.no_grad():
            for p in list(self.model.parameters()) + [self.model.fused.qflat]:
                dist.broadcast(p.data, src=src, group=self.pg)

    # ------------------------------------------------------------------ eager / graph
    def eager_step(self, y, traj):
        vals = self._forward_backward(y, traj)
        self._allreduce()
        self._update()
        return vals

    def _gather(self):
        """pool rows of the static index buffer, both tensors in one native launch"""
        from bcnf_amd import _native as N
        sidx = self._static[2]
        py, pt = self._pool
        n = sidx.shape[0]
        y = torch.empty((n,) + tuple(py.shape[1:]), dtype=py.dtype, device=py.device)
        t = torch.empty((n,) + tuple(pt.shape[1:]), dtype=pt.dtype, device=pt.device)
        cy = py[0].numel() if py.shape[0] else 1
        ct = pt[0].numel() if pt.shape[0] else 1
        N.check(N.lib().bcnf_gather_rows2(N.ptr(sidx), n, N.ptr(py), cy, N.ptr(y), N.ptr(pt), ct, N.ptr(t),
                                          N.stream_handle(py.device)), "bcnf_gather_rows2")
        return y, t

    def _snapshot(self):
        with torch.no_grad():
            params = [p.detach().clone() for p in self.model.parameters()]
            opt = {id(p): {k: v.clone() for k, v in st.items() if torch.is_tensor(v)}
                   for p, st in self.opt.state.items()}
            rng = self.model.fused.rng_state().clone()
        return params, opt, rng

    def _restore(self, snap):
        params, opt, rng = snap
        with torch.no_grad():
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
        self._static = (y.clone(), traj.clone(), None if idx is None else idx.clone())
        sy, st, _ = self._static
        indexed = idx is not None
        snap = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                if indexed:
                    sy, st = self._gather()
                self.eager_step(sy, st)
            self._restore(snap)
        torch.cuda.current_stream().wait_stream(s)
        self.opt.zero_grad(set_to_none=True)
        # the three logged values land in pinned host memory as the graph's last node: the host reads
        # them after one stream sync instead of issuing a separate device-to-host copy per step
        self._host_vals = torch.empty(3, dtype=torch.float32, pin_memory=True)
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            if indexed:
                sy, st = self._gather()
            vals = self._forward_backward(sy, st)
            if self.world == 1:
                self._update()
                self._host_vals.copy_(vals, non_blocking=True)
        g2 = None
        if self.world > 1:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._update()
                self._host_vals.copy_(vals, non_blocking=True)
        self._graphs = (g1, g2, vals)

    def step(self, y, traj):
        """One training step; returns (loss, nll, mse) as Python floats (the Trainer's three .item())."""
        vals = self.step_async(y, traj)
        if not self.capture:
            return tuple(vals.tolist())
        return self._host_values()

    def _host_values(self):
        torch.cuda.current_stream().synchronize()
        return tuple(self._host_vals.tolist())

    def step_async(self, y, traj):
        if not self.capture:
            return self.eager_step(y, traj)
        if self._graphs is None:
            self._build_graphs(y, traj)
        sy, st, _ = self._static
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
        self._pool = (y_pool, traj_pool)

    def step_indexed(self, idx):
        """step(pool_y[idx], pool_traj[idx]) with the gather captured in the graph."""
        if self._pool is None:
            raise RuntimeError("step_indexed() needs set_pool()")
        idx = idx.to(dtype=torch.int64).contiguous()
        if not self.capture:
            self._static = (None, None, idx)
            return tuple(self.eager_step(*self._gather()).tolist())
        if self._graphs is None:
            py, pt = self._pool
            self._build_graphs(py.index_select(0, idx), pt.index_select(0, idx), idx=idx)
        self._static[2].copy_(idx, non_blocking=True)
        self._replay()
        return self._host_values()

    def _replay(self):
        g1, g2, vals = self._graphs
        g1.replay()
        if g2 is not None:
            self._allreduce()
            g2.replay()
        return vals


__all__ = ["TrainStep", "FusedAdam", "clip_grad_norm_"]

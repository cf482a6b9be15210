"""Trainer-semantics training step on the fused stack, with HIP-graph capture and data parallelism.

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

MI355X specifics: the coupling-stack parameters are ONE flat leaf (model.flat_parameters()), so Adam,
the clip and the all-reduce each touch one contiguous buffer; the whole step is captured once into a
HIP graph and replayed (for world > 1 the collective runs between two captured segments).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from bcnf_amd.utils import inn_nll_loss


def _make_adam(params, lr, capturable):
    kw = dict(lr=lr, capturable=capturable)
    try:
        return torch.optim.Adam(params, fused=True, **kw)
    except (RuntimeError, TypeError, ValueError):
        return torch.optim.Adam(params, foreach=True, **kw)


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
        self.opt = _make_adam(self.params, lr, capturable=capture)
        self.mse = torch.nn.MSELoss()
        self._graphs = None
        self._static = None

    # ------------------------------------------------------------------ step pieces
    def _forward_backward(self, y, traj):
        self.opt.zero_grad(set_to_none=True)
        z, h = self.model(y, traj, log_det_J=True, return_features=True)
        nll = inn_nll_loss(z, self.model.log_det_J)
        if self.hybrid_weight > 0:
            mse = self.mse(self.model.prediction_head(h), y)
        else:
            mse = torch.zeros((), device=y.device)
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
        torch.nn.utils.clip_grad_norm_(self.params, max_norm=self.max_norm, foreach=True)

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

    def _build_graphs(self, y, traj, warmup: int = 3):
        self._static = (y.clone(), traj.clone())
        sy, st = self._static
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.eager_step(sy, st)
        torch.cuda.current_stream().wait_stream(s)
        self.opt.zero_grad(set_to_none=True)
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            vals = self._forward_backward(sy, st)
            if self.world == 1:
                self._update()
        g2 = None
        if self.world > 1:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._update()
        self._graphs = (g1, g2, vals)

    def step(self, y, traj):
        """One training step; returns (loss, nll, mse) as Python floats (the Trainer's three .item())."""
        vals = self.step_async(y, traj)
        return tuple(vals.tolist())

    def step_async(self, y, traj):
        if not self.capture:
            return self.eager_step(y, traj)
        if self._graphs is None:
            self._build_graphs(y, traj)
        sy, st = self._static
        sy.copy_(y, non_blocking=True)
        st.copy_(traj, non_blocking=True)
        g1, g2, vals = self._graphs
        g1.replay()
        if g2 is not None:
            self._allreduce()
            g2.replay()
        return vals

"""Which NLL path does TrainStep take on the bench's FC_large model? (counts the wide-fold / plain launches)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bcnf_amd import CondRealNVP_v2, cnf  # noqa: E402
from bcnf_amd.data import DeviceBatches  # noqa: E402
from bcnf_amd.train import TrainStep  # noqa: E402

calls = {"fold": 0, "plain": 0}
f0, s0 = cnf.stack_nll_wide_fold, cnf.stack_nll


def fold(*a, **k):
    calls["fold"] += 1
    return f0(*a, **k)


def plain(*a, **k):
    calls["plain"] += 1
    return s0(*a, **k)


cnf.stack_nll_wide_fold, cnf.stack_nll = fold, plain
dev = torch.device("cuda")
model = CondRealNVP_v2.from_config(bench.FC_LARGE).to(dev).train()
data = DeviceBatches(16384, 2048, dev, seed=1)
idx = data.next_indices()
y, traj = data.y[idx], data.traj[idx]
print("types", type(model.fused).__name__, y.dtype, traj.dtype, traj.shape, y.requires_grad)
print("wide_fold", model._wide_fold(y, (traj,)) is not None)
fns = list(model.feature_network_stack.feature_networks)
print([type(f).__name__ for f in fns], [type(m).__name__ for m in fns[1].nn][-3:])
step = TrainStep(model, lr=2e-4, capture=True)
step.set_pool(data.y, data.traj)
step.set_epoch(torch.cat([data.next_indices() for _ in range(4)]), 2048)
step.run_epoch(2)
print("calls", calls, "cond_shape", step._cond_shape)

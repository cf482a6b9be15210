"""Data-parallel TrainStep on the GPU box with two ranks sharing cuda:0 over gloo (the 8-GPU RCCL run is the
driver's): the captured HIP-graph step, the single gradient bucket and its all-reduce between the two graph
segments. Two ranks with batches b0, b1 (dropout off) must end a step with identical parameters, equal to one
single-process step on the union batch (the mean of per-rank mean gradients is the union's mean gradient)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = {"global": {"parameter_selection": [str(i) for i in range(19)]},
       "model": {"kwargs": {"size": 19, "nested_sizes": [16] * 3, "n_conditions": 80, "n_blocks": 4,
                            "dropout": 0.0, "act_norm": True}},
       "feature_networks": [{"type": "ConcatenateCondition", "kwargs": {"input_size": None, "output_size": 90}},
                            {"type": "FullyConnected", "kwargs": {"sizes": [90, 80]}}]}
WIDE = {"global": CFG["global"], "feature_networks": CFG["feature_networks"],
        "model": {"kwargs": {"size": 19, "nested_sizes": [48] * 2, "n_conditions": 80, "n_blocks": 3,
                             "dropout": 0.0, "act_norm": True}}}


STEPS = 3      # run_epoch at world 2: g1, then (all-reduce, merged update + next step) twice, then the last update


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(n=64):
    g = torch.Generator().manual_seed(3)
    return torch.randn(2 * n, 19, generator=g), torch.randn(2 * n, 30, 3, generator=g)


def _model(cfg):
    from bcnf_amd import CondRealNVP_v2
    torch.manual_seed(11)
    return CondRealNVP_v2.from_config(cfg).cuda().train()


def _worker(rank, world, port, cfg, q, mode="step"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import traceback
    try:
        from bcnf_amd.train import TrainStep
        m = _model(cfg)
        step = TrainStep(m, lr=1e-3, capture=True)
        step.broadcast_parameters()
        y, t = _data()
        n = y.shape[0] // world
        if mode == "epoch":     # bench.py's N > 1 path: device pool, epoch order, run_epoch (gather in the graph)
            step.set_pool(y[rank * n:(rank + 1) * n].cuda(), t[rank * n:(rank + 1) * n].cuda())
            step.set_epoch(torch.arange(n, device="cuda").repeat(STEPS), n)
            logged = step.run_epoch()
            # the logged (loss, nll, mse) of every step == those of the same steps through step()
            m2 = _model(cfg)
            s2 = TrainStep(m2, lr=1e-3, capture=True)
            s2.broadcast_parameters()
            ref = [s2.step(y[rank * n:(rank + 1) * n].cuda(), t[rank * n:(rank + 1) * n].cuda()) for _ in range(STEPS)]
            assert logged == ref, (logged, ref)
        else:
            for _ in range(STEPS):
                step.step(y[rank * n:(rank + 1) * n].cuda(), t[rank * n:(rank + 1) * n].cuda())
        q.put((rank, ([p.detach().cpu().numpy() for p in m.parameters()], step._packed_inplace)))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["step", "epoch"])
@pytest.mark.parametrize("cfg", [CFG, WIDE], ids=["small_family", "wide_family"])
def test_two_rank_step_equals_union_batch_step(cfg, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
        res[r], inplace = res[r]
        # the folded backward (small family) writes its gradients into the all-reduce bucket: no copy
        assert inplace == (cfg is CFG)
    from bcnf_amd.train import TrainStep
    m = _model(cfg)
    step = TrainStep(m, lr=1e-3, capture=True)
    y, t = _data()
    for _ in range(STEPS):
        step.step(y.cuda(), t.cuda())
    ref = [p.detach().cpu() for p in m.parameters()]
    for a, b, c in zip(res[0], res[1], ref):
        a, b = torch.from_numpy(a), torch.from_numpy(b)
        assert torch.equal(a, b)                                  # replicas stay identical
        assert torch.allclose(a, c, rtol=1e-4, atol=1e-6), float((a - c).abs().max())

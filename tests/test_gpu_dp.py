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
        step = TrainStep(m, lr=1e-3, capture=True, overlap_ranges=2 if mode == "overlap" else 0)
        if mode == "overlap":   # wide family: eager steps, the coupling gradient all-reduced in 2 block ranges
            assert step.overlap_ranges == 2 and not step.capture
        step.broadcast_parameters()
        y, t = _data()
        n = y.shape[0] // world
        if mode == "diverge":   # only rank 1's shard of batch 1 blows up; the global loss decides, on both ranks
            yl, tl = y[rank * n:(rank + 1) * n].clone(), t[rank * n:(rank + 1) * n]
            step.set_pool(torch.cat([yl, yl * (1e4 if rank == 1 else 1.0)]).cuda(), torch.cat([tl, tl]).cuda())
            order = torch.cat([torch.arange(n), torch.arange(n) + n, torch.arange(n), torch.arange(n)])
            step.set_epoch(order.cuda(), n)
            from bcnf_amd.train import TrainingDivergedError
            try:
                step.run_epoch(check_divergence=True)
                raised = None
            except TrainingDivergedError as e:
                raised = str(e)
            q.put((rank, ([p.detach().cpu().numpy() for p in m.parameters()],
                          (raised, step._host_cursor, int(step._epoch[1].item())))))
            return
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


@pytest.mark.parametrize("mode,cfg", [("step", CFG), ("epoch", CFG), ("step", WIDE), ("epoch", WIDE),
                                      ("overlap", WIDE)],
                         ids=["small_step", "small_epoch", "wide_step", "wide_epoch", "wide_overlap_ranges"])
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


def test_two_rank_divergence_halts_every_rank_on_the_same_step():
    """One rank's shard diverges (local NLL ~1e8, the other's is normal): the divergence guard judges the
    all-reduced loss, so BOTH ranks raise at the same batch, with the same cursor and identical parameters (no rank
    left blocked in a later all-reduce)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, CFG, q, "diverge")) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    (p0, st0), (p1, st1) = res[0], res[1]
    assert st0 == st1, (st0, st1)
    assert st0[0] is not None and "at batch 1" in st0[0] and st0[1] == 2 and st0[2] == 2
    for a, b in zip(p0, p1):
        assert (a == b).all()

"""Data-parallel plumbing of TrainStep on CPU with the gloo backend, world_size 2.

The HIP kernels need a GPU; these tests cover what is rank-dependent: the one-time parameter broadcast
(rank 0's RNG-seeded init, frozen orthonormal matrices included, must win on every rank) and the
gradient all-reduce (sum / world) that TrainStep runs between its two captured graph segments.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import FC_SMALL_CFG


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import traceback
    try:
        torch.set_num_threads(1)
        from bcnf_amd import CondRealNVP_v2
        from bcnf_amd.train import TrainStep
        torch.manual_seed(1000 + rank)                      # different init per rank on purpose
        m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
        step = TrainStep(m, capture=False)
        assert step.world == world
        step.broadcast_parameters()
        sd = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
        # gradients: rank r holds (r + 1) * base  ->  mean = base * (world + 1) / 2
        for i, p in enumerate(step.params):
            p.grad = torch.full_like(p, float(rank + 1)) * (i + 1)
        step._allreduce()
        grads = [p.grad.detach().numpy().copy() for p in step.params]
        q.put((rank, sd, grads))               # numpy: no shared-memory handles outliving the worker
    except Exception:
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_broadcast_and_allreduce_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, sd, grads = q.get(timeout=240)
        assert grads is not None, sd
        out[rank] = ({k: torch.from_numpy(v) for k, v in sd.items()}, [torch.from_numpy(g) for g in grads])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0, g0 = out[0]
    sd1, g1 = out[1]
    assert sd0.keys() == sd1.keys()
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k                # rank 0's parameters everywhere
    torch.manual_seed(1000)
    from bcnf_amd import CondRealNVP_v2
    ref = CondRealNVP_v2.from_config(FC_SMALL_CFG).state_dict()
    for k in sd0:
        assert torch.equal(sd0[k], ref[k]), k
    for i, (a, b) in enumerate(zip(g0, g1)):
        expect = torch.full_like(a, (1 + 2) / 2 * (i + 1))
        assert torch.equal(a, b) and torch.allclose(a, expect)


def _overlap_worker(rank, world, port, q):
    """The overlapped exchange of the wide family (TrainStep.overlap_ranges): slices of the bucket all-reduced
    asynchronously while the backward runs (WideStack.on_range -> _reduce_range), then the rest of the bucket and a
    join (_reduce_bucket). Here the backward's writes are simulated on CPU: every gradient is a view of the bucket."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import traceback
    try:
        torch.set_num_threads(1)
        from bcnf_amd import CondRealNVP_v2
        from bcnf_amd.train import TrainStep
        m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
        step = TrainStep(m, capture=False)
        for p in step.params:
            p.grad = torch.zeros_like(p)
        step._allreduce()                                    # allocates the bucket; .grad become its views
        n = step._bucket.numel()
        vals = torch.tensor([1.0 + rank, 2.0, 3.0])
        for i, p in enumerate(step.params):                  # rank r holds (r + 1) * (i + 1) * ramp
            p.grad.copy_(torch.linspace(0, 1, p.numel()).view_as(p) * float((rank + 1) * (i + 1)))
        # two "finished ranges" handed over out of order, one of them ending inside a parameter tensor
        step._reduce_range(n // 2, n - 50)
        step._reduce_range(7, n // 3)
        assert len(step._works) == 2
        out = step._allreduce(vals)
        assert not step._works and not step._reduced
        res = [p.grad.detach().numpy().copy() for p in step.params]
        # a step that raised after handing a slice over: the next step joins and forgets it first (_drain_slices)
        step._reduce_range(0, 10)
        step._drain_slices()
        assert not step._works and not step._reduced
        # the stack hooks live only around a step's own backward, also when it raises
        step._hooks = {"on_range": step._reduce_range, "range_blocks": [(0, 1)]}
        with pytest.raises(ZeroDivisionError):
            with step._stack_hooks():
                assert m.fused.on_range is not None and m.fused.range_blocks == [(0, 1)]
                1 / 0
        assert m.fused.on_range is None and m.fused.range_blocks is None
        q.put((rank, res, out.detach().numpy().copy(),
               step._packed_inplace))
    except Exception:
        q.put((rank, traceback.format_exc(), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_overlapped_slice_allreduce_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, grads, vals, inplace = q.get(timeout=240)
        assert vals is not None, grads
        out[rank] = (grads, vals, inplace)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (g0, v0, i0), (g1, v1, i1) = out[0], out[1]
    assert i0 and i1                                          # every gradient was already in its bucket slot
    for i, (a, b) in enumerate(zip(g0, g1)):
        a, b = torch.from_numpy(a), torch.from_numpy(b)
        expect = torch.linspace(0, 1, a.numel()).view_as(a) * ((1 + 2) / 2 * (i + 1))
        assert torch.equal(a, b) and torch.allclose(a, expect, rtol=1e-6, atol=1e-7), i
    assert (v0 == v1).all() and abs(v0[0] - 1.5) < 1e-6      # logged values averaged with the gradients

"""Sharded posterior sampling (bcnf_amd/sampling.py; BASELINE configs[4], SURVEY §8e "replicas plus independent
shards"): shard arithmetic and the gather on CPU (gloo, world size 2 and 3); the draw itself against the oracle on
the GPU (same z, tiled conditions as CondRealNVP_v2._sample(outer=True), cnf.py:572-582)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import FC_SMALL_CFG, close, golden_sd
from oracle import cnf_oracle as O


@pytest.mark.parametrize("n", [0, 1, 5, 1024, 1023])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    from bcnf_amd.sampling import shard_range
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 == a1
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_sampler(c):
    # deterministic per condition: draw s of condition row c -> c.sum() * (s + 1) in every coordinate
    s = torch.arange(1, 4, dtype=torch.float32).view(3, 1, 1)
    return (c.sum(dim=(1, 2)).view(1, -1, 1) * s).expand(3, c.shape[0], 19).contiguous()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bcnf_amd.sampling import draw_sharded
        import bench
        cond = torch.arange(7 * 30 * 3, dtype=torch.float32).view(7, 30, 3)
        # bench.py's sampling spin-up shape: time-bounded, so the ranks run it a different number of times -- it must
        # hold no collective, or the gathered call below would pair up with a spin-up call of another rank
        bench.spinup(lambda: draw_sharded(None, 3, cond, sampler=_fake_sampler, gather=False), 20 + 40 * rank)
        out = draw_sharded(None, 3, cond, sampler=_fake_sampler)
        local = draw_sharded(None, 3, cond, sampler=_fake_sampler, gather=False)
        q.put((rank, torch.equal(out, _fake_sampler(cond)), tuple(local.shape)))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_draw_sharded_gathers_every_condition_once(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    from bcnf_amd.sampling import shard_range
    for rank, ok, shape in res:
        assert ok is True, ok
        a, b = shard_range(7, rank, world)
        assert shape == (3, b - a, 19)


@pytest.mark.gpu
def test_draw_matches_oracle_tiled_inverse(g1):
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.sampling import draw
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
    m.load_state_dict(golden_sd(g1))
    m.to("cuda").eval()
    sd = golden_sd(g1)
    gen = torch.Generator().manual_seed(9)
    cond = torch.randn(37, 30, 3, generator=gen)
    n = 11
    z = torch.randn(n * 37, 19, generator=gen)
    got = draw(m, n, cond.cuda(), z=z.cuda()).cpu()
    h = O.feature_forward(sd, O.FC_SMALL_SPEC, cond.repeat(n, 1, 1))       # cnf.py:579 tiling
    ref = O.model_inverse(sd, O.FC_SMALL_SPEC, z, h).view(n, 37, 19)
    ok, err = close(got, ref)
    assert ok, err
    # device z stream: shape, determinism under a seeded generator
    g = torch.Generator(device="cuda").manual_seed(5)
    a = draw(m, 4, cond.cuda(), generator=g)
    g = torch.Generator(device="cuda").manual_seed(5)
    b = draw(m, 4, cond.cuda(), generator=g)
    assert a.shape == (4, 37, 19) and torch.equal(a, b)


@pytest.mark.gpu
def test_config4_launch_rows_match_small_launch_and_oracle(g1):
    """configs[4] at its launch shape: ONE draw over all 1024 conditions x 500 draws; the rows of 8 conditions are
    bit-identical to a small launch over just those conditions (the row -> condition map and the 16-row MFMA tiles
    mix no rows), and match the oracle's tiled inverse at the 1e-5 gate."""
    from bcnf_amd import CondRealNVP_v2
    from bcnf_amd.sampling import draw
    torch.manual_seed(0)
    m = CondRealNVP_v2.from_config(FC_SMALL_CFG)
    m.load_state_dict(golden_sd(g1))
    m.to("cuda").eval()
    sd = golden_sd(g1)
    gen = torch.Generator().manual_seed(41)
    n, N = 500, 1024
    cond = torch.randn(N, 30, 3, generator=gen)
    z = torch.randn(n * N, 19, generator=gen)
    full = draw(m, n, cond.cuda(), z=z.cuda()).cpu()
    assert full.shape == (n, N, 19)
    cols = torch.tensor([0, 1, 146, 511, 512, 877, 1022, 1023])
    zs = z.view(n, N, 19)[:, cols].reshape(-1, 19)
    small = draw(m, n, cond[cols].cuda(), z=zs.cuda()).cpu()
    assert torch.equal(full[:, cols], small)
    h = O.feature_forward(sd, O.FC_SMALL_SPEC, cond[cols])
    ref = O.model_inverse(sd, O.FC_SMALL_SPEC, zs, h.repeat(n, 1)).view(n, len(cols), 19)
    ok, err = close(full[:, cols], ref)
    assert ok, err

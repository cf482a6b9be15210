"""Posterior sampling at scale (BASELINE.json configs[4]: 500 draws per condition x 1024 conditions, 1 -> 8 GPUs).

`CondRealNVP_v2.sample` keeps the reference's semantics (cnf.py:510-588: CPU-generator z stream, chunking by
batch_size / sample_batch_size, output on `output_device`). For throughput, `draw` produces the same (n, N, D)
layout as `sample(n, cond, outer=True)` (row s * N + i = draw s of condition i, cnf.py:577-582) without the
reference's chunking: the feature network runs once per condition, z is drawn on the device (torch's
counter-based generator, seedable), and the inverse runs as ONE launch sequence over all n * N rows with the
row -> condition map (`cond_index`), so the tiled features are never materialised.

`draw_sharded` splits the conditions over the ranks of a process group: every rank holds a replica of the model
and samples its own contiguous slice of conditions, with no collective on the data path ("replicas
plus independent shards"); the only exchange is the final all-gather of the shards.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) slice of n items for `rank`; the first n % world ranks get one extra item."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


@torch.no_grad()
def draw(model, n_samples: int, *conditions: torch.Tensor, sigma: float = 1.0,
         generator: torch.Generator | None = None, z: torch.Tensor | None = None) -> torch.Tensor:
    """n_samples posterior draws for each of the N conditions: (n_samples, N, D) on the model's device.
    `z` (n_samples * N, D), row s * N + i, replaces the device draw (parity tests)."""
    h = model.feature_network_stack(*conditions).contiguous()       # once per condition
    nc = h.shape[0]
    D = model.size
    if n_samples == 0 or nc == 0:
        return torch.empty((n_samples, nc, D), dtype=torch.float32, device=h.device)
    if z is None:
        z = torch.randn(n_samples * nc, D, device=h.device, generator=generator)
    else:
        z = z.to(device=h.device, dtype=torch.float32).contiguous().clone()
    if sigma != 1.0:
        z.mul_(sigma)
    idx = torch.arange(n_samples * nc, device=h.device, dtype=torch.int64) % nc
    return model._inverse_indexed(z, h, idx).view(n_samples, nc, D)


@torch.no_grad()
def draw_sharded(model, n_samples: int, conditions: torch.Tensor, group=None, gather: bool = True,
                 sampler: Callable | None = None, **kwargs) -> torch.Tensor:
    """`draw` over all N conditions with the conditions sharded across the ranks of `group` (contiguous slices,
    shard_range). Returns the full (n_samples, N, D) on every rank when gather=True, else the local
    (n_samples, N_local, D). `sampler(cond_slice) -> (n_samples, n_local, D)` replaces `draw` (tests)."""
    world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
    rank = dist.get_rank(group) if world > 1 else 0
    n = conditions.shape[0]
    a, b = shard_range(n, rank, world)
    local_c = conditions[a:b]
    if sampler is None:
        local = draw(model, n_samples, local_c, **kwargs)
    else:
        local = sampler(local_c)
    if world == 1 or not gather:
        return local
    # equal-size buffers for all_gather: pad every shard to the largest one
    width = n // world + (1 if n % world else 0)
    D = local.shape[-1]
    buf = torch.empty((world, n_samples, width, D), dtype=local.dtype, device=local.device)
    mine = torch.zeros((n_samples, width, D), dtype=local.dtype, device=local.device)
    mine[:, : b - a] = local
    dist.all_gather(list(buf.unbind(0)), mine, group=group)
    parts = []
    for r in range(world):
        ra, rb = shard_range(n, r, world)
        parts.append(buf[r, :, : rb - ra])
    return torch.cat(parts, dim=1)


__all__ = ["shard_range", "draw", "draw_sharded"]

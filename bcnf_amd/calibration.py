"""Calibration ranks (psaegert/bcnf src/bcnf/eval/calibration.py:20-48) with the counting on the GPU.

`compute_y_hat_ranks` keeps the reference's signature and result: ranks[i, d] = #{draws s : y_hat[s, i, d] < y[i, d]}
(int64, (N, D), on `output_device`). The posterior draws come from the HIP inverse; the count is
`bcnf_rank_count` (bcnf_amd/csrc/bcnf_eval.hip), which accumulates chunk by chunk.

z_stream = "reference" (default): the draws are CondRealNVP_v2.sample(outer=True, batch_size, sample_batch_size),
i.e. the reference's CPU-generator z stream and chunking, so the ranks equal the reference's for the same seed.
z_stream = "device": draws are generated on the GPU (`bcnf_amd.sampling.draw`, seedable `generator`) in chunks of
`chunk_draws` and counted as they are produced; the (M, N, D) tensor of all draws is never materialised.

Deviation: the reference moves the model to `device` (default 'cpu'); the HIP kernels need the GPU, so a CPU
`device` keeps the model where it is (it must already be on a ROCm device).
"""
from __future__ import annotations

import torch

from bcnf_amd import _native as N


def rank_count_(counts: torch.Tensor, y_hat: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """counts (N, D) uint32-as-int32 device tensor += #{s : y_hat[s] < y} for y_hat (M, N, D) and y (N, D)."""
    if y_hat.dim() != 3 or y.dim() != 2 or y_hat.shape[1:] != y.shape or counts.shape != y.shape:
        raise ValueError(f"rank_count_: shapes {tuple(y_hat.shape)}, {tuple(y.shape)}, {tuple(counts.shape)}")
    for t in (y_hat, y, counts):
        if not t.is_cuda:
            raise RuntimeError("bcnf_amd rank counting runs on the GPU only")
    y_hat = y_hat.to(torch.float32).contiguous()
    y = y.to(torch.float32).contiguous()
    N.check(N.lib().bcnf_rank_count(N.ptr(y_hat), N.ptr(y), y_hat.shape[0], y.shape[0], y.shape[1], N.ptr(counts),
                                    N.stream_handle(y.device)), "bcnf_rank_count")
    return counts


@torch.no_grad()
def compute_y_hat_ranks(model, y: torch.Tensor, *conditions: torch.Tensor, M_samples: int = 10_000,
                        batch_size: int = 100, sample_batch_size: int | None = None, device: str = "cpu",
                        output_device: str = "cpu", verbose: bool = True, z_stream: str = "reference",
                        generator: torch.Generator | None = None, chunk_draws: int = 500) -> torch.Tensor:
    if sample_batch_size is None:
        sample_batch_size = batch_size
    if torch.device(device).type != "cpu":
        model.to(device)
    model.eval()
    dev = model.fused.flat.device
    if dev.type != "cuda":
        raise RuntimeError("bcnf_amd compute_y_hat_ranks: the model must be on a ROCm device")
    y_dev = y.to(dev, torch.float32)
    counts = torch.zeros(y_dev.shape, dtype=torch.int32, device=dev)
    if z_stream == "reference":
        y_hat = model.sample(M_samples, *conditions, outer=True, batch_size=batch_size,
                             sample_batch_size=sample_batch_size, output_device=dev, verbose=verbose)
        rank_count_(counts, y_hat, y_dev)
    elif z_stream == "device":
        from bcnf_amd.sampling import draw
        conds = [c.to(dev) for c in conditions]
        done = 0
        while done < M_samples:
            m = min(chunk_draws, M_samples - done)
            rank_count_(counts, draw(model, m, *conds, generator=generator), y_dev)
            done += m
    else:
        raise ValueError(f"z_stream must be 'reference' or 'device', got {z_stream!r}")
    return counts.to(torch.int64).to(output_device)


__all__ = ["compute_y_hat_ranks", "rank_count_"]

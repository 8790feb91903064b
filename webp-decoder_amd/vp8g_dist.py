"""vp8g_dist -- the (tiny) multi-GPU layer of the batch decoder.

Independent frames shard with no data-path collective: each rank owns a
contiguous shard of the global batch, builds its own device-resident inputs and launches its own
kernel.  The only exchanges are small and off the timed path:

  * share_frame_params   -- broadcast rank 0's per-frame parameter blocks (Vp8gFrameDesc:
                            dequant factors + loop-filter table, 176 B per frame), so every rank
                            decodes with identical tables;
  * gather_frame_digests -- all-gather one 64-bit digest per checked frame (never pixels: 512 x
                            12.4 MB per GPU would cost more link time than the kernels);
  * reduce_timing        -- max over ranks of wall / kernel time, min of the parity flags.

Works with any torch.distributed backend: "nccl" (= RCCL over xGMI) on the GPU node, "gloo" in
the CPU tests (tests/test_dist.py).  One process per GPU, launched by torch.distributed.run.
"""
from __future__ import annotations

import torch


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) frame range of `rank`; sizes differ by at most one frame."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def share_frame_params(desc_bytes: torch.Tensor, dist) -> torch.Tensor:
    """Broadcast rank 0's descriptor block (uint8 tensor, same shape on all ranks) in place."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(desc_bytes, src=0)
    return desc_bytes


def gather_frame_digests(digests: torch.Tensor, dist) -> torch.Tensor:
    """All-gather per-rank int64 digest vectors (equal length) -> [world, n] tensor."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return digests.unsqueeze(0)
    out = [torch.empty_like(digests) for _ in range(dist.get_world_size())]
    dist.all_gather(out, digests)
    return torch.stack(out)


def reduce_timing(elapsed_s: float, kernel_ms: float, ok: bool, dist, device) -> tuple[float, float, bool]:
    """(max wall seconds, max kernel ms, all ranks bit-exact)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed_s, kernel_ms, ok
    t = torch.tensor([elapsed_s, kernel_ms, 0.0 if ok else 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1]), bool(t[2] < 0.5)


def digest64(data: bytes) -> int:
    """First 8 bytes of sha256 as a signed int64 (fits an int64 tensor for all_gather)."""
    import hashlib
    return int.from_bytes(hashlib.sha256(data).digest()[:8], "little", signed=True)

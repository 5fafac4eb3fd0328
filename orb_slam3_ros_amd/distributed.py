"""Multi-GPU batching: frames are sharded one-shard-per-GPU (weak scaling, no data-path
collective during extraction) and the resulting per-image feature slots are exchanged with ONE
all-gather so every rank (every tracking thread of a multi-camera rig, BASELINE config 4) sees
every stream's keypoints + descriptors. Over RCCL ("nccl" backend) this is the xGMI all-gather of
SURVEY.md §8(e); the same code runs over gloo for the CPU tests.

Slot layout per image (fixed size so the collective needs no size exchange):
  int32[2] {n, monoIndex} | cv::KeyPoint[cap] (7 x 4 B) | uint8[cap][32] descriptors.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> range:
    """Contiguous block of frame indices owned by `rank` (frame f -> rank f * world // n_total)."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return range(start, start + base + (1 if rank < rem else 0))


def slot_bytes(cap: int) -> int:
    return 8 + cap * 28 + cap * 32


def pack_slots(counts: torch.Tensor, kps: torch.Tensor, desc: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """counts [n,2] i32, kps [n,cap,7] i32, desc [n,cap,32] u8 -> out [n, slot_bytes] u8."""
    n, cap = kps.shape[0], kps.shape[1]
    out[:, 0:8].copy_(counts.contiguous().view(torch.uint8).view(n, 8))
    out[:, 8:8 + 28 * cap].copy_(kps.contiguous().view(torch.uint8).view(n, 28 * cap))
    out[:, 8 + 28 * cap:].copy_(desc.contiguous().view(n, 32 * cap))
    return out


def unpack_slots(buf: torch.Tensor, cap: int):
    n = buf.shape[0]
    counts = buf[:, 0:8].contiguous().view(torch.int32).view(n, 2)
    kps = buf[:, 8:8 + 28 * cap].contiguous().view(torch.int32).view(n, cap, 7)
    desc = buf[:, 8 + 28 * cap:].contiguous().view(n, cap, 32)
    return counts, kps, desc


def allgather_slots(local: torch.Tensor, gathered: torch.Tensor | None = None, group=None) -> torch.Tensor:
    """All-gather equal-size [n, slot] u8 blocks from every rank -> [world*n, slot]."""
    world = dist.get_world_size(group)
    if gathered is None:
        gathered = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        parts = list(gathered.chunk(world, 0))
        dist.all_gather(parts, local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(gathered, local.contiguous(), group=group)
    return gathered

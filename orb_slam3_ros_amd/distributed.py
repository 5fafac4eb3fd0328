"""Multi-GPU batching: frames are sharded one-shard-per-GPU (weak scaling, no data-path
collective during extraction) and the resulting per-image feature slots are exchanged with ONE
all-gather so every rank (every tracking thread of a multi-camera rig, BASELINE config 4) sees
every stream's keypoints + descriptors. Over RCCL ("nccl" backend) this is the xGMI all-gather of
SURVEY.md §8(e); the same code runs over gloo for the CPU tests.

Slot layout per image (fixed size so the collective needs no size exchange):
  int32[2] {n, monoIndex} | cv::KeyPoint[cap] (7 x 4 B) | uint8[cap][32] descriptors.

Slab layout (the zero-copy form the bench uses): the extractor writes its batch outputs straight
into one flat buffer per step, [counts int32[n][2] | keypoints int32[n][cap][7] | descriptors
u8[n][cap][32]], so the all-gather moves that buffer as is (no pack kernels) and the gathered
tensor is world slabs back to back. SlabExchange double-buffers the slabs and issues the gather
asynchronously, so step k's exchange over xGMI runs under step k+1's kernels.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> range:
    """Contiguous block of frame indices owned by `rank`; the first n_total % world ranks take one extra."""
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


def slab_bytes(n_img: int, cap: int) -> int:
    return n_img * (8 + cap * 28 + cap * 32)


def slab_views(buf: torch.Tensor, n_img: int, cap: int):
    """(counts [n,2] i32, kps [n,cap,7] i32, desc [n,cap,32] u8) views of a flat u8 slab."""
    assert buf.dtype == torch.uint8 and buf.dim() == 1 and buf.numel() == slab_bytes(n_img, cap)
    o1 = 8 * n_img
    o2 = o1 + 28 * cap * n_img
    counts = buf[:o1].view(torch.int32).view(n_img, 2)
    kps = buf[o1:o2].view(torch.int32).view(n_img, cap, 7)
    desc = buf[o2:].view(n_img, cap, 32)
    return counts, kps, desc


class SlabExchange:
    """Double-buffered slab all-gather. Step k writes slab k % 2 (bind its views as the extractor's
    outputs), then post(k) gathers it without blocking the stream order of the next step; before
    slab k % 2 is rewritten two steps later, acquire(k) makes the current stream wait for that
    slab's gather. gloo (CPU rehearsal) gathers host copies synchronously."""

    def __init__(self, n_img: int, cap: int, device, group=None, buffers: int = 2):
        self.n, self.cap, self.group = n_img, cap, group
        self.world = dist.get_world_size(group)
        self.gloo = dist.get_backend(group) == "gloo"
        nb = slab_bytes(n_img, cap)
        self.local = [torch.zeros(nb, dtype=torch.uint8, device=device) for _ in range(buffers)]
        gdev = "cpu" if self.gloo else device
        self.gathered = [torch.zeros(self.world * nb, dtype=torch.uint8, device=gdev) for _ in range(buffers)]
        self.pending = [None] * buffers

    def views(self, k: int):
        return slab_views(self.local[k % len(self.local)], self.n, self.cap)

    def acquire(self, k: int):
        i = k % len(self.local)
        if self.pending[i] is not None:
            self.pending[i].wait()
            self.pending[i] = None

    def post(self, k: int):
        i = k % len(self.local)
        if self.gloo:
            parts = list(self.gathered[i].chunk(self.world))
            dist.all_gather(parts, self.local[i].cpu(), group=self.group)
        else:
            self.pending[i] = dist.all_gather_into_tensor(self.gathered[i], self.local[i], group=self.group,
                                                          async_op=True)

    def drain(self):
        for i in range(len(self.pending)):
            if self.pending[i] is not None:
                self.pending[i].wait()
                self.pending[i] = None

    def rank_views(self, k: int, r: int):
        """(counts, kps, desc) of rank r in the gathered slab of step k (after drain/acquire)."""
        nb = slab_bytes(self.n, self.cap)
        g = self.gathered[k % len(self.gathered)]
        return slab_views(g[r * nb:(r + 1) * nb], self.n, self.cap)

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


def rig_role(rank: int) -> tuple[int, int]:
    """BASELINE config 4 over 2 x streams ranks (one image per GPU): stream s's
    left camera on rank 2s, its right camera on rank 2s + 1. Returns (stream, camera)."""
    return rank // 2, rank % 2


class StereoRigExchange:
    """Config 4's multi-GPU layout (TUM-VI KannalaBrandt8 stereo, Frame.cc:1034-1166): each rank
    extracts its camera of its stream for K consecutive frames per step (one launch, vLappingArea
    `lap`), the step's slots are all-gathered once (K steps of one image batched per collective,
    SURVEY.md §8(e)), and the left-camera rank runs ComputeStereoFishEyeMatches' descriptor stage
    (knnMatch k=2 + ratio over the lapping rows, Frame.cc:1126-1151) for those K frames against the
    right-camera slots its partner rank produced (orbfe_stereo_knn_slabs). Every rank ends a step
    holding every stream's keypoints and descriptors (the gathered slab).

    Step k writes slab k % 2; match(k) makes the caller's stream wait for step k's gather and
    enqueues the kNN, so calling match(k - 1) after extract(k) overlaps the gather with the next
    step's kernels. gloo (CPU rehearsal) exchanges host copies synchronously. Every launch goes to
    the caller's current torch stream (the default stream is handle 0 = the legacy null stream,
    which the C-ABI takes as such), so the gather that post(k) orders after that stream sees the
    finished slab (tests/test_distributed.py::test_rig_exchange_gpu_gloo checks every step)."""

    def __init__(self, K: int, width: int, height: int, nfeatures: int = 1000, lap=(0, 511), ratio: float = 0.7,
                 device=None, group=None):
        import ctypes

        from . import _lib
        self.lib, self._lib = _lib.load(), _lib
        self.K, self.W, self.H = int(K), int(width), int(height)
        self.lap, self.ratio = (int(lap[0]), int(lap[1])), float(ratio)
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if self.world % 2:
            raise ValueError("config 4's rig layout needs an even number of ranks (two cameras per stream)")
        self.stream_id, self.camera = rig_role(self.rank)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        h = ctypes.c_void_p()
        _lib.check(self.lib.orbfe_extractor_create(nfeatures, 1.2, 8, 20, 7, ctypes.byref(h)), "create")
        self.h = h
        self.cap = _lib.check(self.lib.orbfe_extractor_capacity(h, self.W, self.H), "capacity")
        self.xchg = SlabExchange(self.K, self.cap, self.device, group)
        self.l2r = torch.full((self.K, self.cap), -1, dtype=torch.int32, device=self.device)
        self.dist = torch.full((self.K, self.cap), -1, dtype=torch.int32, device=self.device)
        self.ngood = torch.zeros(self.K, dtype=torch.int32, device=self.device)
        self._ptr_key, self._ptrs = None, None
        self._partner = None   # gloo: device copy of the partner's gathered slab

    def extract(self, images, k: int):
        """images: [K, H, W] u8 device tensor, this rank's camera for the step's K frames."""
        import ctypes
        assert images.shape == (self.K, self.H, self.W) and images.dtype == torch.uint8 and images.is_cuda
        self.xchg.acquire(k)
        counts, kps, desc = self.xchg.views(k)
        _ = self._lib.check(self.lib.orbfe_set_batch_outputs(self.h, kps.data_ptr(), desc.data_ptr(),
                                                             counts.data_ptr(), self.K), "set_batch_outputs")
        key = (images.data_ptr(), images.stride(0))
        if key != self._ptr_key:
            self._ptrs = (ctypes.c_void_p * self.K)(*[images.data_ptr() + i * images.stride(0) for i in range(self.K)])
            self._ptr_key = key
        s = torch.cuda.current_stream(self.device).cuda_stream
        self._lib.check(self.lib.orbfe_extract_batch(self.h, self.K, self._ptrs, self.W, self.H, images.stride(1),
                                                     self.lap[0], self.lap[1], s), "extract_batch")
        self.xchg.post(k)

    def match(self, k: int):
        """Left-camera ranks: the fisheye kNN of step k's K frames (own slab x the partner's gathered
        slab) into l2r / dist / ngood; right-camera ranks: nothing."""
        i = k % len(self.xchg.local)
        if self.xchg.pending[i] is not None:   # the caller's stream waits for step k's gather
            self.xchg.pending[i].wait()
            self.xchg.pending[i] = None
        if self.camera != 0:
            return
        cl, _, dl = self.xchg.views(k)
        cr, _, dr = self.xchg.rank_views(k, self.rank + 1)
        if cr.device != self.device:   # gloo rehearsal: the gathered slab is a host tensor
            if self._partner is None:
                self._partner = torch.empty(slab_bytes(self.K, self.cap), dtype=torch.uint8, device=self.device)
            nb = slab_bytes(self.K, self.cap)
            g = self.xchg.gathered[i]
            self._partner.copy_(g[(self.rank + 1) * nb:(self.rank + 2) * nb])
            cr, _, dr = slab_views(self._partner, self.K, self.cap)
        s = torch.cuda.current_stream(self.device).cuda_stream
        self._lib.check(self.lib.orbfe_stereo_knn_slabs(cl.data_ptr(), dl.data_ptr(), 0, 1, cr.data_ptr(),
                                                        dr.data_ptr(), 0, 1, self.cap, self.K, self.ratio,
                                                        self.l2r.data_ptr(), self.dist.data_ptr(),
                                                        self.ngood.data_ptr(), s), "stereo_knn_slabs")

    def drain(self):
        self.xchg.drain()

    def close(self):
        if self.h:
            self.lib.orbfe_set_batch_outputs(self.h, None, None, None, 0)
            self.lib.orbfe_extractor_destroy(self.h)
            self.h = None

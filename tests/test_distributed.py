"""CPU (gloo, world_size 2): frame sharding and the per-image feature-slot all-gather used by the
multi-GPU bench path (orb_slam3_ros_amd/distributed.py)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import pytest

from orb_slam3_ros_amd import distributed as odist


def test_shard_range_partitions():
    for n in (1, 7, 256, 1001):
        for w in (1, 2, 3, 8):
            got = [list(odist.shard_range(n, r, w)) for r in range(w)]
            assert sum(got, []) == list(range(n))


def _worker(rank, world, port, cap, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 3
    g = torch.Generator().manual_seed(rank)
    counts = torch.tensor([[rank * 10 + i, i] for i in range(n)], dtype=torch.int32)
    kps = torch.randint(-1000, 1000, (n, cap, 7), dtype=torch.int32, generator=g)
    desc = torch.randint(0, 256, (n, cap, 32), dtype=torch.uint8, generator=g)
    local = odist.pack_slots(counts, kps, desc, torch.empty((n, odist.slot_bytes(cap)), dtype=torch.uint8))
    allb = odist.allgather_slots(local)
    c2, k2, d2 = odist.unpack_slots(allb, cap)
    ok = torch.equal(c2[rank * n:(rank + 1) * n], counts) and torch.equal(k2[rank * n:(rank + 1) * n], kps) and \
        torch.equal(d2[rank * n:(rank + 1) * n], desc)
    ok = ok and all(int(c2[r * n, 0]) == r * 10 for r in range(world))
    out[rank] = 1 if ok else 0
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_allgather_slots_gloo():
    world, cap = 2, 17
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), cap, out), nprocs=world, join=True)
    assert dict(out) == {0: 1, 1: 1}


def _slab_worker(rank, world, port, cap, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 4
    x = odist.SlabExchange(n, cap, "cpu")
    ok = True
    ref = {}
    for k in range(5):   # more steps than buffers: slabs are reused
        x.acquire(k)
        counts, kps, desc = x.views(k)
        g = torch.Generator().manual_seed(100 * k + rank)
        counts.copy_(torch.tensor([[rank * 10 + i, k] for i in range(n)], dtype=torch.int32))
        kps.copy_(torch.randint(-1000, 1000, (n, cap, 7), dtype=torch.int32, generator=g))
        desc.copy_(torch.randint(0, 256, (n, cap, 32), dtype=torch.uint8, generator=g))
        ref[k] = (counts.clone(), kps.clone(), desc.clone())
        x.post(k)
        x.drain()
        for r in range(world):
            c2, k2, d2 = x.rank_views(k, r)
            ok = ok and int(c2[0, 0]) == r * 10 and int(c2[0, 1]) == k
            if r == rank:
                ok = ok and torch.equal(c2, ref[k][0]) and torch.equal(k2, ref[k][1]) and torch.equal(d2, ref[k][2])
    out[rank] = 1 if ok else 0
    dist.destroy_process_group()


def test_slab_layout_views():
    n, cap = 3, 5
    buf = torch.arange(odist.slab_bytes(n, cap), dtype=torch.int64).to(torch.uint8)
    c, k, d = odist.slab_views(buf, n, cap)
    assert c.shape == (n, 2) and k.shape == (n, cap, 7) and d.shape == (n, cap, 32)
    assert c.data_ptr() == buf.data_ptr() and k.data_ptr() == buf.data_ptr() + 8 * n
    assert d.data_ptr() + d.numel() == buf.data_ptr() + buf.numel()


def test_slab_exchange_gloo():
    world, cap = 2, 9
    out = mp.Manager().dict()
    mp.spawn(_slab_worker, args=(world, _free_port(), cap, out), nprocs=world, join=True)
    assert dict(out) == {0: 1, 1: 1}


def _oracle_frames(ids, cap):
    """Real ORB output of synthetic frames (the CPU oracle stands in for the GPU extractor here):
    counts [n,2] = (N, monoIndex), keypoints [n,cap,7] (cv::KeyPoint records), descriptors."""
    import numpy as np
    from oracle import oracle
    from orb_slam3_ros_amd.synth import synth_image
    ex = oracle.OracleExtractor(500, 1.2, 8, 20, 7)
    counts = torch.zeros((len(ids), 2), dtype=torch.int32)
    kps = torch.zeros((len(ids), cap, 7), dtype=torch.int32)
    desc = torch.zeros((len(ids), cap, 32), dtype=torch.uint8)
    for i, f in enumerate(ids):
        mono, k, d = ex(synth_image(1000 + f, 376, 240), (0, 1000))
        n = len(k)
        assert 0 < n <= cap
        counts[i] = torch.tensor([n, mono], dtype=torch.int32)
        kps[i, :n] = torch.from_numpy(np.ascontiguousarray(k).view(np.int32).reshape(n, 7).copy())
        desc[i, :n] = torch.from_numpy(d)
    ex.close()
    return counts, kps, desc


def _real_worker(rank, world, port, nframes, cap, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = odist.shard_range(nframes, rank, world)
    c, k, d = _oracle_frames(list(mine), cap)
    local = odist.pack_slots(c, k, d, torch.empty((len(mine), odist.slot_bytes(cap)), dtype=torch.uint8))
    c2, k2, d2 = odist.unpack_slots(odist.allgather_slots(local), cap)
    # every rank sees every frame's features, in frame order, identical to extracting it locally
    rc, rk, rd = _oracle_frames(list(range(nframes)), cap)
    out[rank] = int(torch.equal(c2, rc) and torch.equal(k2, rk) and torch.equal(d2, rd))
    dist.destroy_process_group()


def test_allgather_real_features_gloo():
    """The all-gather of SURVEY §8(e) on real extractor output (not random bytes): frames sharded
    over 2 ranks by shard_range, slots packed, gathered and unpacked bit-exactly."""
    from oracle import oracle
    oracle.build()
    world, nframes, cap = 2, 4, 600
    out = mp.Manager().dict()
    mp.spawn(_real_worker, args=(world, _free_port(), nframes, cap, out), nprocs=world, join=True)
    assert dict(out) == {0: 1, 1: 1}


def _rig_frames(stream, K):
    """K consecutive synthetic TUM-VI-like 512x512 stereo pairs of one stream (seeded by stream)."""
    from orb_slam3_ros_amd.synth import synth_stereo
    return [synth_stereo(5000 + 100 * stream + f, 512, 512) for f in range(K)]


def _rig_worker(rank, world, port, K, cap, out):
    """BASELINE config 4's layout on the CPU: each rank extracts its camera of its stream (the oracle
    stands in for the device extractor), the slabs are all-gathered, and the left rank runs the
    fisheye kNN + ratio on its own slots against the partner's gathered ones."""
    import numpy as np
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stream, cam = odist.rig_role(rank)
    frames = _rig_frames(stream, K)
    ex = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    x = odist.SlabExchange(K, cap, "cpu")
    counts, kps, desc = x.views(0)
    for f, pair in enumerate(frames):
        mono, k, d = ex(pair[cam], (0, 511))
        n = len(k)
        counts[f] = torch.tensor([n, mono], dtype=torch.int32)
        kps[f, :n] = torch.from_numpy(np.ascontiguousarray(k).view(np.int32).reshape(n, 7).copy())
        desc[f, :n] = torch.from_numpy(d)
    x.post(0)
    x.drain()
    ok = True
    if cam == 0:
        cr, _, dr = x.rank_views(0, rank + 1)
        exr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
        for f, (left, right) in enumerate(frames):
            ml, nl = int(counts[f, 1]), int(counts[f, 0])
            mr, nr = int(cr[f, 1]), int(cr[f, 0])
            g, t, dd = oracle.stereo_knn_ratio(desc[f, ml:nl].numpy(), dr[f, mr:nr].numpy(), 0.7)
            omr, _, odr = exr(right, (0, 511))
            oml, _, odl = ex(left, (0, 511))
            g2, t2, d2 = oracle.stereo_knn_ratio(odl[oml:], odr[omr:], 0.7)
            ok = ok and g == g2 and np.array_equal(t, t2) and np.array_equal(dd, d2) and g > 0
    out[rank] = int(ok)
    dist.destroy_process_group()


def test_rig_layout_gloo():
    """Config 4 over 2 ranks (one stream: left camera on rank 0, right on rank 1): the right camera's
    slots reach the left rank through the slab all-gather intact, and the kNN there equals the one
    computed from both images directly."""
    from oracle import oracle
    oracle.build()
    assert [odist.rig_role(r) for r in range(4)] == [(0, 0), (0, 1), (1, 0), (1, 1)]
    world, K, cap = 2, 2, 1100
    out = mp.Manager().dict()
    mp.spawn(_rig_worker, args=(world, _free_port(), K, cap, out), nprocs=world, join=True)
    assert dict(out) == {0: 1, 1: 1}


def _rig_gpu_worker(rank, world, port, K, steps, out):
    import numpy as np
    from oracle import oracle
    from orb_slam3_ros_amd.synth import synth_stereo
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stream, cam = odist.rig_role(rank)
    # a distinct stereo pair for every (step, frame): a wrong slab index, or a gather overwritten by
    # a later extraction, shows up as another step's kNN
    frames = [[synth_stereo(7000 + 1000 * k + 100 * stream + f, 512, 512) for f in range(K)] for k in range(steps)]
    imgs = [torch.from_numpy(np.stack([p[cam] for p in fr])).cuda() for fr in frames]
    rig = odist.StereoRigExchange(K, 512, 512, device=torch.device("cuda", 0))
    got = []

    def take():
        torch.cuda.synchronize()
        got.append((rig.l2r.cpu().numpy().copy(), rig.ngood.cpu().numpy().copy()))

    for k in range(steps):   # steps >= 3: slabs 0 and 1 are both reused, the match lagging one step
        rig.extract(imgs[k], k)
        if k:
            rig.match(k - 1)
            take()
    rig.match(steps - 1)
    rig.drain()
    take()
    ok = True
    if cam == 0:
        for k in range(steps):
            l2r, ngood = got[k]
            for f, (left, right) in enumerate(frames[k]):
                ol, orr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
                ml, kl, dl = ol(left, (0, 511))
                mr, kr, dr = orr(right, (0, 511))
                g, t, _ = oracle.stereo_knn_ratio(dl[ml:], dr[mr:], 0.7)
                exp = np.full(rig.cap, -1, np.int32)
                exp[ml:len(kl)][t >= 0] = t[t >= 0] + mr
                ok = ok and int(ngood[f]) == g and np.array_equal(l2r[f], exp)
    rig.close()
    out[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rig_exchange_gpu_gloo():
    """StereoRigExchange (config 4's multi-GPU layout) with two ranks sharing cuda:0 over gloo: every
    step's (distinct images, both slabs reused) batched kNN on the left rank, from the partner's
    gathered slots, read right after that step's match, is bit-exact against the oracle."""
    from oracle import oracle
    oracle.build()
    world, K, steps = 2, 2, 4
    out = mp.Manager().dict()
    mp.spawn(_rig_gpu_worker, args=(world, _free_port(), K, steps, out), nprocs=world, join=True)
    assert dict(out) == {0: 1, 1: 1}

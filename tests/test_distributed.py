"""CPU (gloo, world_size 2): frame sharding and the per-image feature-slot all-gather used by the
multi-GPU bench path (orb_slam3_ros_amd/distributed.py)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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

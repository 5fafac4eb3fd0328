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

"""GPU diagnostic: the strengthened rig-exchange test with per-step / per-frame reporting (which step,
which frame, counts and kNN vs the oracle). usage: python tools/rig_diag.py"""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros_amd import distributed as odist  # noqa: E402


def worker(rank, world, port, K, steps, sync_each):
    from oracle import oracle
    from orb_slam3_ros_amd.synth import synth_stereo
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stream, cam = odist.rig_role(rank)
    frames = [[synth_stereo(7000 + 1000 * k + 100 * stream + f, 512, 512) for f in range(K)] for k in range(steps)]
    imgs = [torch.from_numpy(np.stack([p[cam] for p in fr])).cuda() for fr in frames]
    rig = odist.StereoRigExchange(K, 512, 512, device=torch.device("cuda", 0))
    got, cnt = [], []

    def take(k):
        torch.cuda.synchronize()
        got.append((rig.l2r.cpu().numpy().copy(), rig.ngood.cpu().numpy().copy()))
        cl, _, _ = rig.xchg.views(k)
        cr, _, _ = rig.xchg.rank_views(k, rank + 1 if cam == 0 else rank)
        cnt.append((cl.cpu().numpy().copy(), cr.cpu().numpy().copy()))

    for k in range(steps):
        rig.extract(imgs[k], k)
        if sync_each:
            torch.cuda.synchronize()
        if k:
            rig.match(k - 1)
            take(k - 1)
    rig.match(steps - 1)
    rig.drain()
    take(steps - 1)
    if cam == 0:
        for k in range(steps):
            l2r, ngood = got[k]
            cl, cr = cnt[k]
            for f, (left, right) in enumerate(frames[k]):
                ol, orr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
                ml, kl, dl = ol(left, (0, 511))
                mr, kr, dr = orr(right, (0, 511))
                g, t, _ = oracle.stereo_knn_ratio(dl[ml:], dr[mr:], 0.7)
                exp = np.full(rig.cap, -1, np.int32)
                exp[ml:len(kl)][t >= 0] = t[t >= 0] + mr
                bad = int((l2r[f] != exp).sum())
                print(f"step {k} frame {f}: left counts gpu {tuple(cl[f])} oracle {(len(kl), ml)}; right counts gpu "
                      f"{tuple(cr[f])} oracle {(len(kr), mr)}; ngood gpu {int(ngood[f])} oracle {g}; l2r mismatches {bad}",
                      flush=True)
    rig.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    from oracle import oracle
    oracle.build()
    for sync_each in (False, True):
        s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
        print("sync_each", sync_each, flush=True)
        mp.spawn(worker, args=(2, port, 2, 4, sync_each), nprocs=2, join=True)

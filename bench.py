#!/usr/bin/env python3
"""bench.py — ORB front-end throughput on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one batch of synthetic stereo frames resident in HBM:
ORBextractor::operator() on every left and right image (pyramid, FAST cells, octree,
orientation, blur, rBRIEF) + Frame::ComputeStereoMatches per frame, all on the GPU (liborbfe.so).
With N > 1 GPUs (torchrun, one process per GPU) every rank processes its own shard of frames
(weak scaling) and each step's keypoint + descriptor slab is all-gathered over RCCL, overlapped
with the next step's kernels (distributed.SlabExchange); the timed region ends after the last
step's gather.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline bytes.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match (752×480, 1000 kp) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Algorithmic bytes of the pyramid+FAST pass per 752x480 image: every level read
# once + levels 1..7 written once.
PYR_FAST_BYTES = {(752, 480): 1873774, (1241, 376): 2421578, (512, 512): 1361776}


def level_sizes(w, h, nlevels=8, sf=1.2):
    s = [np.float32(1.0)]
    for i in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(sf))))
    inv = [np.float32(1.0) / v for v in s]
    return [(int(np.rint(np.float32(w) * v)), int(np.rint(np.float32(h) * v))) for v in inv]


def algorithmic_bytes(w, h):
    lv = level_sizes(w, h)
    return sum(a * b for a, b in lv) + sum(a * b for a, b in lv[1:])


def pmc_traffic(n_img, w, h):
    """HBM bytes per pyramid+FAST pass from the newest committed PMC summary for this workload
    (profiles/rNN_pmc_traffic.json, written by tools/pmc_summary.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this same bench command); None when there is none."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("images_per_step"), d.get("width"), d.get("height")) == (n_img, w, h):
            best = (d["pyramid_fast_traffic_bytes_per_step"], os.path.basename(f))
    return best


def pmc_cache(n_img, w, h):
    """Descriptor-pass L2 hit rate and LDS bank-conflict share from the newest committed cache PMC
    summary for this workload (profiles/rNN_pmc_cache.json, tools/pmc_cache_summary.py)."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_cache.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("images_per_step"), d.get("width"), d.get("height")) == (n_img, w, h):
            best = (d["kernels"], os.path.basename(f))
    return best


def copy_peak_gbps(torch, dev, nbytes=1 << 30, reps=10):
    """Measured device-to-device copy rate (read + write bytes / time) of a 1 GiB buffer with the
    library's 16-byte-per-lane streaming copy kernel: the practical HBM ceiling the roofline is
    also quoted against."""
    from orb_slam3_ros_amd import _lib
    lib = _lib.load()
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream(dev)

    def cp():
        _lib.check(lib.orbfe_copy_stream(a.data_ptr(), b.data_ptr(), nbytes, s.cuda_stream), "copy_stream")

    cp()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        cp()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def cpu_baseline(pairs_l, pairs_r, w, h, nfeatures, bf, fx):
    """Oracle CPU path (C++ restatement, kind='port') on a bounded sample, host cores."""
    from oracle import oracle
    oracle.build()
    L = oracle.lib()
    threads = max(1, min(16, os.cpu_count() or 1))
    # bounded sample: about 10 s wall on 16 threads (the oracle needs ~40 ms per stereo frame per core)
    n = min(max(400, 250 * threads), 4000)
    idx = [i % len(pairs_l) for i in range(n)]
    Ls = np.ascontiguousarray(np.stack([pairs_l[i] for i in idx]))
    Rs = np.ascontiguousarray(np.stack([pairs_r[i] for i in idx]))
    t0 = time.perf_counter()
    L.oro_bench_stereo(Ls.ctypes.data, Rs.ctypes.data, n, w, h, nfeatures, 1.2, 8, 20, 7, bf, fx, threads)
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(n / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} stereo frames {w}x{h} (extract L+R + ComputeStereoMatches), {threads} threads, "
                      f"frame-parallel, oracle/orb_oracle.cpp -O3 -march=x86-64-v3; host CPU: {cpu}",
            "seconds": round(dt, 3)}


def matcher_config5(steps):
    """BASELINE config 5: SearchByProjection(Frame&, local map) of 100k synthetic map points against
    a 1000-keypoint stereo frame, seed 12345, th in {1, 3, 5, 15}, nnratio 0.8 (Tracking.cc:3429).
    Timed through the host C-ABI call (records packed + uploaded every call, result copied back)."""
    from orb_slam3_ros_amd import synth_match as sm
    from orb_slam3_ros_amd.matcher import ORBmatcher
    rng = np.random.default_rng(12345)
    F = sm.synth_frame(rng, 1000)
    mps = sm.synth_local_map(rng, F, 100_000)
    mvp0, obs = sm.initial_slots(rng, F.N)
    m = ORBmatcher(0.8)
    lib = m._lib
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device
    dev_t = torch.device("cuda", torch.cuda.current_device())
    Fd = DeviceMatchFrame(F, dev_t)
    obs_t = torch.from_numpy(obs.copy()).to(dev_t)
    mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(dev_t)
    out = {}
    for th in (1, 3, 5, 15):
        for _ in range(2):
            m.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, th)
        bufs = [mvp0.copy() for _ in range(steps)]
        t0 = time.perf_counter()
        for b in bufs:
            n = m.SearchByProjectionLocalMap(F, b, obs, mps, th)
        dt = (time.perf_counter() - t0) / steps
        # device time of the kernels alone (records already uploaded), HIP events on the call's stream
        lib.orbfe_matcher_set_timing(1)
        dev = []
        for _ in range(steps):
            m.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, th)
            dev.append(lib.orbfe_matcher_last_ms())
        lib.orbfe_matcher_set_timing(0)
        dms = float(np.mean(dev))
        # device-resident call (records, slots and frame already in HBM): wall time per call, which
        # includes the host-checked convergence of the ordered passes
        mvp_t = [torch.from_numpy(mvp0.copy()).to(dev_t) for _ in range(steps + 2)]
        for b in mvp_t[:2]:
            search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in mvp_t[2:]:
            nd = search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
        torch.cuda.synchronize()
        rdt = (time.perf_counter() - t0) / steps
        assert nd == n
        out[f"th{th}"] = {"ms_per_call": round(dt * 1e3, 4), "calls_per_s": round(1.0 / dt, 2),
                          "queries_per_s": round(len(mps) / dt, 1), "device_ms_per_call": round(dms, 4),
                          "device_queries_per_s": round(len(mps) / (dms * 1e-3), 1),
                          "resident_ms_per_call": round(rdt * 1e3, 4),
                          "resident_queries_per_s": round(len(mps) / rdt, 1), "nmatches": int(n)}
    # Tracking::SearchLocalPoints' projection (isInFrustum + PredictScale) fused with the
    # th=1 search, 100k world points, device time (HIP events)
    from orb_slam3_ros_amd.matcher import search_local_points
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, 100_000)
    lib.orbfe_matcher_set_timing(1)
    dev = []
    for _ in range(steps + 2):
        nm, ntm = search_local_points(F, cam, pts, mvp0.copy(), obs, 1.0)
        dev.append(lib.orbfe_matcher_last_ms())
    lib.orbfe_matcher_set_timing(0)
    dms = float(np.mean(dev[2:]))
    out["search_local_points_th1"] = {"device_ms_per_call": round(dms, 4), "points": len(pts), "n_to_match": ntm,
                                      "nmatches": int(nm), "device_points_per_s": round(len(pts) / (dms * 1e-3), 1)}
    return {"workload": "SearchByProjection local map: 100k map points (30% noisy copies, Binomial(256,0.05) "
                        "flips) vs 1000-keypoint stereo frame, nnratio 0.8, seed 12345",
            "timing": "ms_per_call: host C-ABI call incl. 8 MB record upload and result download; "
                      "device_ms_per_call: kernels only (grid build, ordered passes, commit), HIP events; "
                      "resident_ms_per_call: orbfe_search_by_projection_local_device wall time with the "
                      "records, slots and frame already in HBM",
            "per_th": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=256, help="stereo frames per GPU per step")
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--unique", type=int, default=16, help="distinct synthetic frames (tiled over the batch)")
    ap.add_argument("--pipelines", type=int, default=1, help="sub-batches on separate HIP streams")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stage-steps", type=int, default=10, help="extra steps with per-stage HIP events")
    ap.add_argument("--matcher-steps", type=int, default=10, help="config-5 SearchByProjection calls per th (0: skip)")
    ap.add_argument("--rectify-steps", type=int, default=5,
                    help="time cv::remap rectification of the step's images (reported separately; 0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the measured path); gloo = CPU rehearsal of the multi-rank path")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses cuda:0 (rehearse N ranks on a 1-GPU box with --dist-backend gloo)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    from orb_slam3_ros_amd.synth import synth_stereo
    from orb_slam3_ros_amd import distributed as odist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    W, H, F = args.width, args.height, args.frames
    bf, fx = 0.110078 * 458.654, 458.654   # EuRoC stereo baseline x fx
    U = min(args.unique, F)
    pairs = [synth_stereo(1000 * rank + i, W, H) for i in range(U)]
    host = np.empty((2 * F, H, W), np.uint8)
    for f in range(F):
        host[2 * f], host[2 * f + 1] = pairs[f % U]
    images = torch.from_numpy(host).to(dev)
    fe = StereoFrontEnd(F, W, H, nfeatures=args.nfeatures, bf=bf, fx=fx, device=dev, pipelines=args.pipelines)
    gather = world > 1 and not args.no_allgather
    if gather:
        # zero-copy, double-buffered slab exchange: the extractor writes step k's outputs into slab
        # k % 2 and its all-gather runs asynchronously under step k + 1's kernels
        xchg = odist.SlabExchange(2 * F, fe.cap, dev)
    it = [0]

    def step():
        k = it[0]
        it[0] += 1
        if gather:
            xchg.acquire(k)             # the gather that last read slab k % 2 has finished
            fe.bind_outputs(*xchg.views(k))
        fe.run(images)
        if gather:
            xchg.post(k)

    def drain():
        if gather:
            xchg.drain()

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()                             # every step's exchange is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cpu" if gloo else dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * F * args.steps / elapsed

    # per-stage HIP-event timing on the launch stream (separate steps, same workload, one pipeline
    # so the events bracket kernels that run alone on the GPU)
    fe_t = fe if args.pipelines == 1 else StereoFrontEnd(F, W, H, nfeatures=args.nfeatures, bf=bf, fx=fx, device=dev)
    fe_t.set_stage_timing(True)
    for _ in range(args.stage_steps):
        fe_t.run(images)
    torch.cuda.synchronize()
    stages, nrec = fe_t.stage_timing()
    fe_t.set_stage_timing(False)
    if fe_t is not fe:
        fe_t.close()
    rect = None
    if args.rectify_steps > 0 and rank == 0:
        # System::TrackStereo's cv::remap of every image before extraction (not part of
        # `value`: the reference's metric starts at the rectified images)
        from orb_slam3_ros_amd.rectify import rectify_maps, remap_linear_batch
        mx, my = rectify_maps(W, H, fx, 457.296, W / 2 - 8.6, H / 2 + 8.4, (-0.28340811, 0.07395907, 0.00019359, 1.76e-05))
        dmx, dmy = torch.from_numpy(mx).to(dev), torch.from_numpy(my).to(dev)
        rout = torch.empty_like(images)
        remap_linear_batch(images, dmx, dmy, rout)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.rectify_steps):
            remap_linear_batch(images, dmx, dmy, rout)
        e1.record()
        torch.cuda.synchronize()
        rms = e0.elapsed_time(e1) / args.rectify_steps
        rbytes = images.numel() * (1 + 1) + 2 * 4 * W * H   # read + write per image, maps once (L2 / IC)
        rect = {"ms_per_step": round(rms, 4), "images": int(images.shape[0]),
                "achieved_GBps": round(rbytes / (rms * 1e-3) / 1e9, 1)}
        del rout
    counts = fe.counts.cpu().numpy()
    nm = fe.nmatch.cpu().numpy()

    if rank == 0:
        n_img = 2 * F
        pyr_fast_ms = stages["resize"] + stages["fast"]
        bytes_img = algorithmic_bytes(W, H)
        achieved = n_img * bytes_img / (pyr_fast_ms * 1e-3) / 1e9 if pyr_fast_ms > 0 else 0.0
        dominant = max(stages, key=stages.get)
        tr = pmc_traffic(n_img, W, H)
        cache = pmc_cache(n_img, W, H)
        copy_peak = copy_peak_gbps(torch, dev)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": "EuRoC-MH01-like stereo 752x480 (BASELINE config 2): ORBextractor L+R "
                            "(nFeatures=%d, scale 1.2, 8 levels, FAST 20/7) + ComputeStereoMatches" % args.nfeatures,
                "frames_per_gpu_per_step": F,
                "images_per_gpu_per_step": 2 * F,
                "width": W, "height": H,
                "allgather": gather,
                "allgather_backend": (args.dist_backend if gather else None),
                "allgather_bytes_per_rank_per_step": (odist.slab_bytes(2 * F, fe.cap) if gather else 0),
                "allgather_overlap": (None if not gather else "synchronous host copies (gloo rehearsal)" if gloo else
                                      "async, double-buffered: step k's gather runs under step k+1's kernels"),
                "pipelines": args.pipelines,
                "parallelism": f"frame-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "pyramid+FAST pass (k_resize x7 + k_fast)",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": tr[0] if tr else None,
                "traffic_unit": "bytes per launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": tr[1] if tr else None,
                "bytes_per_image": bytes_img,
                "images_per_launch": n_img,
                "kernel_ms_per_launch": round(pyr_fast_ms, 4),
                "copy_peak_measured": round(copy_peak, 1),
                "frac_vs_copy_peak": round(achieved / copy_peak, 4),
            },
            "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            "dominant_stage": dominant,
            "keypoints_per_image_mean": float(counts[:, 0].mean()),
            "stereo_matches_per_frame_mean": float(nm.mean()),
        }
        if cache is not None and "k_describe" in cache[0]:
            kd = cache[0]["k_describe"]
            result["describe_pass"] = {"kernel": "k_describe", "l2_hit_rate": kd["l2_hit_rate"],
                                       "lds_bank_conflict_share": kd["lds_conflict_share"], "source": cache[1]}
        if rect is not None:
            result["rectify_remap"] = rect
        if args.matcher_steps > 0:
            result["matcher_config5"] = matcher_config5(args.matcher_steps)
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline([p[0] for p in pairs], [p[1] for p in pairs], W, H,
                                                  args.nfeatures, bf, fx)
        print(json.dumps(result), flush=True)
    fe.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

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
import ctypes
import datetime
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match (752×480, 1000 kp) at 1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Algorithmic bytes of the pyramid+FAST pass per 752x480 image: every level read
# once + levels 1..7 written once.
PYR_FAST_BYTES = {(752, 480): 1873774, (1241, 376): 2421578, (512, 512): 1361776}
EUROC_BF, EUROC_FX = 0.110078 * 458.654, 458.654   # EuRoC MH_01 stereo: baseline x fx
KITTI_BF, KITTI_FX = 0.5327 * 721.5377, 721.5377   # KITTI 2011_09_26 stereo
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2   # wave64 VALU instr/s: 1024 SIMD-32s, 2 cycles each (MI355X_MICROARCH.md)


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
    (profiles/rNN_pmc_traffic.json, written by tools/pmc_round.py from rocprofv3 FETCH_SIZE /
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


def tr_kernels(n_img, w, h):
    """Per-kernel entries of the newest committed PMC traffic summary of this workload ({} if none)."""
    import glob
    best = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("images_per_step"), d.get("width"), d.get("height")) == (n_img, w, h):
            best = d["kernels"]
    return best


def pmc_cache(n_img, w, h):
    """Descriptor-pass L2 hit rate and LDS bank-conflict share from the newest committed cache PMC
    summary for this workload (profiles/rNN_pmc_cache.json, tools/pmc_round.py)."""
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


def _host_cpu():
    """nproc, the job's usable CPUs (affinity mask, cgroup quota) and lscpu's model / sockets."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def start_native_oracle_build():
    """The reference builds with -O3 -march=native (CMakeLists.txt:11-14): compile the oracle's
    extractor + stereo restatement for THIS host in the background (a few seconds) while the GPU
    legs run. Returns (process, path) or (None, None)."""
    out = os.path.join(tempfile.gettempdir(), f"orbfe_oracle_native_{os.getpid()}.so")
    srcs = [os.path.join(ROOT, "oracle", f) for f in ("orb_oracle.cpp", "orb_oracle_match.cpp", "orb_oracle_bench.cpp")]
    cmd = ["g++", "-O3", "-march=native", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-fPIC", "-shared",
           "-o", out] + srcs + ["-lpthread"]
    try:
        return subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE), out
    except OSError:
        return None, None


def _oracle_cdll(native):
    """The -march=native oracle if it built, else the portable (x86-64-v3) checker build."""
    import ctypes
    from oracle import oracle
    proc, path = native
    flags = "-O3 -march=x86-64-v3 (portable oracle build; the native build failed)"
    L = None
    if proc is not None:
        proc.wait()
        if proc.returncode == 0 and os.path.exists(path):
            L = ctypes.CDLL(path)
            flags = "-O3 -march=native -ffp-contract=off (built on this host at bench time)"
    if L is None:
        oracle.build()
        L = ctypes.CDLL(oracle.LIB)
    vp, ci, cf, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.POINTER(ctypes.c_double)
    L.oro_bench_stereo.restype = ctypes.c_long
    L.oro_bench_stereo.argtypes = [vp, vp, ci, ci, ci, ci, cf, ci, ci, ci, cf, cf, ci]
    L.oro_bench_stereo_latency.restype = ctypes.c_long
    L.oro_bench_stereo_latency.argtypes = [vp, vp, ci, ci, ci, ci, cf, ci, ci, ci, cf, cf, ci, cd]
    L.oro_bench_mono.restype = ctypes.c_long
    L.oro_bench_mono.argtypes = [vp, ci, ci, ci, ci, cf, ci, ci, ci, ci, ci, ci, cd]
    L.oro_bench_fisheye_latency.restype = ctypes.c_long
    L.oro_bench_fisheye_latency.argtypes = [vp, vp, ci, ci, ci, ci, cf, ci, ci, ci, ci, ci, ci, cd]
    L.oro_bench_fisheye.restype = ctypes.c_long
    L.oro_bench_fisheye.argtypes = [vp, vp, ci, ci, ci, ci, cf, ci, ci, ci, ci, ci, ci, cd]
    oracle._match_sigs(L)
    return L, flags


def cpu_baseline(native, budget_s=4.0):
    """SURVEY §8(d) CPU timing of the oracle (the C++ restatement, kind='port') on this host, in
    the same run: per config, 1-thread frame-serial latency, the reference's 2-thread L/R split
    latency (Frame.cc:122-125, stereo configs), and throughput with one frame per thread on every
    CPU the job may use. Each mode runs a bounded sample of about `budget_s` seconds."""
    import ctypes
    from orb_slam3_ros_amd.synth import synth_image, synth_stereo
    L, flags = _oracle_cdll(native)
    cpu = _host_cpu()
    threads = cpu["affinity"] or 1
    if cpu["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(np.ceil(cpu["cgroup_cpu_quota"]))))
    ms = ctypes.c_double()
    out = {}

    def stereo_cfg(name, W, H, nf, bf, fx, seed):
        U = 8
        pairs = [synth_stereo(seed + i, W, H) for i in range(U)]
        Ls = np.ascontiguousarray(np.stack([p[0] for p in pairs]))
        Rs = np.ascontiguousarray(np.stack([p[1] for p in pairs]))
        L.oro_bench_stereo_latency(Ls.ctypes.data, Rs.ctypes.data, 1, W, H, nf, 1.2, 8, 20, 7, bf, fx, 0, ctypes.byref(ms))
        est = max(ms.value, 1.0)
        n1 = int(min(400, max(8, budget_s * 1e3 / est)))
        idx = [i % U for i in range(n1)]
        Ln, Rn = np.ascontiguousarray(Ls[idx]), np.ascontiguousarray(Rs[idx])
        L.oro_bench_stereo_latency(Ln.ctypes.data, Rn.ctypes.data, n1, W, H, nf, 1.2, 8, 20, 7, bf, fx, 0,
                                   ctypes.byref(ms))
        lat1 = ms.value
        L.oro_bench_stereo_latency(Ln.ctypes.data, Rn.ctypes.data, n1, W, H, nf, 1.2, 8, 20, 7, bf, fx, 1,
                                   ctypes.byref(ms))
        lat2 = ms.value
        nt = int(min(20000, max(2 * threads, budget_s * 1e3 * threads / est)))
        idx = [i % U for i in range(nt)]
        Ln, Rn = np.ascontiguousarray(Ls[idx]), np.ascontiguousarray(Rs[idx])
        t0 = time.perf_counter()
        L.oro_bench_stereo(Ln.ctypes.data, Rn.ctypes.data, nt, W, H, nf, 1.2, 8, 20, 7, bf, fx, threads)
        dt = time.perf_counter() - t0
        out[name] = {"latency_1t_ms": round(lat1, 3), "latency_lr2t_ms": round(lat2, 3),
                     "throughput_frames_per_s": round(nt / dt, 2), "throughput_threads": threads,
                     "sample": f"{n1} frames per latency mode, {nt} frames for throughput ({U} distinct "
                               f"synthetic {W}x{H} pairs, nFeatures {nf}); extract L+R + ComputeStereoMatches"}

    def mono_cfg(name, W, H, nf, seed):
        U = 8
        imgs = np.ascontiguousarray(np.stack([synth_image(seed + i, W, H) for i in range(U)]))
        L.oro_bench_mono(imgs.ctypes.data, 1, W, H, nf, 1.2, 8, 20, 7, 0, 1000, 1, ctypes.byref(ms))
        est = max(ms.value, 1.0)
        n1 = int(min(800, max(8, budget_s * 1e3 / est)))
        idx = [i % U for i in range(n1)]
        In = np.ascontiguousarray(imgs[idx])
        L.oro_bench_mono(In.ctypes.data, n1, W, H, nf, 1.2, 8, 20, 7, 0, 1000, 1, ctypes.byref(ms))
        lat1 = ms.value / n1
        nt = int(min(40000, max(2 * threads, budget_s * 1e3 * threads / est)))
        idx = [i % U for i in range(nt)]
        In = np.ascontiguousarray(imgs[idx])
        L.oro_bench_mono(In.ctypes.data, nt, W, H, nf, 1.2, 8, 20, 7, 0, 1000, threads, ctypes.byref(ms))
        out[name] = {"latency_1t_ms": round(lat1, 3), "throughput_frames_per_s": round(nt / (ms.value * 1e-3), 2),
                     "throughput_threads": threads,
                     "sample": f"{n1} frames latency, {nt} frames throughput ({U} distinct synthetic {W}x{H} "
                               f"images, nFeatures {nf}, vLappingArea {{0, 1000}} as the mono Frame passes)"}

    def fisheye_cfg(name, W, H, nf, lap, seed):
        # BASELINE config 4's per-frame CPU path: ExtractORB L || R (lapping {0, 511}) + the fisheye
        # stereo descriptor stage (knnMatch k=2 + ratio 0.7, Frame.cc:1126-1151)
        U = 8
        pairs = [synth_stereo(seed + i, W, H) for i in range(U)]
        Ls = np.ascontiguousarray(np.stack([p[0] for p in pairs]))
        Rs = np.ascontiguousarray(np.stack([p[1] for p in pairs]))
        L.oro_bench_fisheye_latency(Ls.ctypes.data, Rs.ctypes.data, 1, W, H, nf, 1.2, 8, 20, 7, lap[0], lap[1], 0,
                                    ctypes.byref(ms))
        est = max(ms.value, 1.0)
        n1 = int(min(400, max(8, budget_s * 1e3 / est)))
        idx = [i % U for i in range(n1)]
        Ln, Rn = np.ascontiguousarray(Ls[idx]), np.ascontiguousarray(Rs[idx])
        L.oro_bench_fisheye_latency(Ln.ctypes.data, Rn.ctypes.data, n1, W, H, nf, 1.2, 8, 20, 7, lap[0], lap[1], 0,
                                    ctypes.byref(ms))
        lat1 = ms.value
        L.oro_bench_fisheye_latency(Ln.ctypes.data, Rn.ctypes.data, n1, W, H, nf, 1.2, 8, 20, 7, lap[0], lap[1], 1,
                                    ctypes.byref(ms))
        lat2 = ms.value
        nt = int(min(20000, max(2 * threads, budget_s * 1e3 * threads / est)))
        idx = [i % U for i in range(nt)]
        Ln, Rn = np.ascontiguousarray(Ls[idx]), np.ascontiguousarray(Rs[idx])
        L.oro_bench_fisheye(Ln.ctypes.data, Rn.ctypes.data, nt, W, H, nf, 1.2, 8, 20, 7, lap[0], lap[1], threads,
                            ctypes.byref(ms))
        out[name] = {"latency_1t_ms": round(lat1, 3), "latency_lr2t_ms": round(lat2, 3),
                     "throughput_frames_per_s": round(nt / (ms.value * 1e-3), 2), "throughput_threads": threads,
                     "images_per_s": round(2 * nt / (ms.value * 1e-3), 2),
                     "sample": f"{n1} frames per latency mode, {nt} frames for throughput ({U} distinct synthetic "
                               f"{W}x{H} pairs, nFeatures {nf}, vLappingArea {{{lap[0]},{lap[1]}}}); extract L+R + "
                               f"knnMatch(k=2)+ratio of the lapping rows (TriangulateMatches not timed)"}

    def sbp_config5(n_kp=1000, name="config5_search_by_projection_100k"):
        # BASELINE config 5 on the CPU restatement: the same synthetic frame / 100k map points / slots as
        # matcher_config5 (seed 12345). The search is ordered over the map points (later points see
        # earlier assignments, ORBmatcher.cc:88-90), so the reference runs it on one thread.
        from orb_slam3_ros_amd import synth_match as sm
        rng = np.random.default_rng(12345)
        F = sm.synth_frame(rng, n_kp)
        mps = sm.synth_local_map(rng, F, 100_000)
        mvp0, obs = sm.initial_slots(rng, F.N)
        res = {}
        for th in (1, 3, 5, 15):
            times, n = [], 0
            t_end = time.perf_counter() + budget_s / 4
            while time.perf_counter() < t_end or len(times) < 3:
                mvp = mvp0.copy()
                t0 = time.perf_counter()
                n = L.oro_sbp_local(F.ref(), mvp.ctypes.data, obs.ctypes.data, mps.ctypes.data, len(mps), float(th), 0,
                                    50.0, 0.8)
                times.append(time.perf_counter() - t0)
            m = float(np.median(times))
            res[f"th{th}"] = {"ms_per_call": round(m * 1e3, 3), "queries_per_s": round(len(mps) / m, 1),
                              "calls": len(times), "nmatches": int(n)}
        out[name] = {
            "per_th": res, "threads": 1,
            "sample": f"SearchByProjection(F of {n_kp} keypoints, 100k local map points, th) of the matcher_config5 "
                      "workload (seed 12345), median over >= 3 calls per th; ordered over the points, one thread as "
                      "in the reference"}

    t0 = time.perf_counter()
    stereo_cfg("config2_euroc_stereo_752x480", 752, 480, 1000, EUROC_BF, EUROC_FX, 9000)
    stereo_cfg("config2_euroc_stereo_752x480_nf1200", 752, 480, 1200, EUROC_BF, EUROC_FX, 9050)
    mono_cfg("config1_euroc_mono_752x480", 752, 480, 1000, 9100)
    stereo_cfg("config3_kitti_stereo_1241x376", 1241, 376, 2000, KITTI_BF, KITTI_FX, 9200)
    fisheye_cfg("config4_tumvi_fisheye_512x512", 512, 512, 1000, (0, 511), 9300)
    sbp_config5()
    sbp_config5(5000, "config5_search_by_projection_100k_n5000")
    total = time.perf_counter() - t0
    c2 = out["config2_euroc_stereo_752x480"]
    return {"value": c2["throughput_frames_per_s"], "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "config 2 throughput, one stereo frame per thread on every usable CPU; " + c2["sample"],
            "latency_1t": c2["latency_1t_ms"], "latency_lr2t": c2["latency_lr2t_ms"],
            "throughput_nproc": c2["throughput_frames_per_s"], "configs": out, "host": cpu,
            "build": f"oracle/orb_oracle.cpp {flags}", "seconds": round(total, 2),
            "note": "oracle CPU path (faithful C++ restatement), not OpenCV's SIMD code; threads = min(affinity, "
                    "cgroup quota) — nproc reports the whole machine"}


def parity_check(fe, images_host_pairs, frame_pair, nframes, nfeat, bf, fx, stereo="rectified", lap=(0, 0)):
    """CHECKER, outside every timed region: EVERY frame of the last step (nframes = the whole
    batch by default, so both ends of the launch and everything between) against the CPU oracle's
    output for that frame's input pair (keypoint records, descriptors, monoIndex, uRight / depth
    bits, nmatch or the kNN candidates). The batch tiles U distinct synthetic pairs, so the oracle
    runs U times; every frame's GPU output is compared. Returns (ok, message)."""
    import concurrent.futures as cf
    from oracle import oracle
    oracle.build()

    def ref(p):
        left, right = images_host_pairs[p]
        ol, orr = oracle.OracleExtractor(nfeat, 1.2, 8, 20, 7), oracle.OracleExtractor(nfeat, 1.2, 8, 20, 7)
        r = (ol(left, lap), orr(right, lap))
        if stereo == "rectified":
            r = r + (oracle.stereo_match(ol, orr, r[0][1], r[0][2], r[1][1], r[1][2], bf, fx),)
        else:
            ml, mr = r[0][0], r[1][0]
            r = r + (oracle.stereo_knn_ratio(r[0][2][ml:], r[1][2][mr:], 0.7),)
        return r

    uniq = sorted({int(frame_pair[f]) for f in range(nframes)})
    with cf.ThreadPoolExecutor(8) as ex:
        refs = dict(zip(uniq, ex.map(ref, uniq)))
    # one device -> host copy of the whole batch's outputs
    counts = fe.counts[: 2 * nframes].cpu().numpy()
    kps = fe.kps[: 2 * nframes].cpu().numpy()
    desc = fe.desc[: 2 * nframes].cpu().numpy()
    nmatch = fe.nmatch[:nframes].cpu().numpy()
    if stereo == "rectified":
        ur_all = fe.uright[:nframes].cpu().numpy().view(np.uint32)
        dp_all = fe.depth[:nframes].cpu().numpy().view(np.uint32)
    else:
        l2r_all = fe.l2r[:nframes].cpu().numpy()
    for f in range(nframes):
        r = refs[int(frame_pair[f])]
        for side in (0, 1):
            i = 2 * f + side
            n, mono = int(counts[i, 0]), int(counts[i, 1])
            om, ok_, od = r[side]
            if mono != om or n != len(ok_) or not np.array_equal(kps[i, :n].reshape(-1).view(np.uint32),
                                                                 ok_.view(np.uint32).reshape(-1)) \
                    or not np.array_equal(desc[i, :n], od):
                return False, f"frame {f} side {side}: keypoints / descriptors differ from the oracle"
        n = len(r[0][1])
        if stereo == "rectified":
            ur, dp, nm = r[2]
            if int(nmatch[f]) != nm or not np.array_equal(ur_all[f, :n], ur.view(np.uint32)) \
                    or not np.array_equal(dp_all[f, :n], dp.view(np.uint32)):
                return False, f"frame {f}: ComputeStereoMatches output differs from the oracle"
        else:
            good, t, _ = r[2]
            ml, mr = r[0][0], r[1][0]
            exp = np.full(n, -1, np.int32)
            exp[ml:][t >= 0] = t[t >= 0] + mr
            if int(nmatch[f]) != good or not np.array_equal(l2r_all[f, :n], exp):
                return False, f"frame {f}: fisheye kNN candidates differ from the oracle"
    return True, (f"all {nframes} frames ({2 * nframes} images, frames 0..{nframes - 1} incl. both ends of the "
                  f"launch) bit-exact vs the CPU oracle ({len(uniq)} distinct synthetic pairs tiled over the batch)")


def _matcher_pmc():
    """Committed counters of the config-5 search kernels (tools/gpu_matcher_pmc.sh): per th, the
    VALU issue fraction of the pass kernel."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_matcher.json")), reverse=True):
        if os.path.exists(f):
            with open(f) as fh:
                d = json.load(fh)
            return {k: dict(v, source=os.path.basename(f)) for k, v in d.get("per_th", {}).items()}
    return None


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
    matcher_pmc = _matcher_pmc()
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
        # includes its single host round trip (the ordered passes converge on the device); timed at
        # the C-ABI (the drop-in boundary: arguments prepared, as a C++ caller holds them) and
        # through the Python wrapper (its argument checks and stream lookup added)
        mvp_t = [torch.from_numpy(mvp0.copy()).to(dev_t) for _ in range(steps + 2)]
        for b in mvp_t[:2]:
            search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in mvp_t[2:]:
            nd = search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
        torch.cuda.synchronize()
        wdt = (time.perf_counter() - t0) / steps
        assert nd == n
        st = torch.cuda.current_stream(dev_t).cuda_stream
        args = [(Fd.ref(), b.data_ptr(), obs_t.data_ptr(), mps_t.data_ptr(), len(mps), float(th), 0, 50.0, 0.8, st)
                for b in mvp_t[2:]]
        for b in mvp_t[2:]:
            b.copy_(mvp_t[0].new_tensor(mvp0))
        torch.cuda.synchronize()
        fn = lib.orbfe_search_by_projection_local_device
        t0 = time.perf_counter()
        for a in args:
            nd = fn(*a)
        torch.cuda.synchronize()
        rdt = (time.perf_counter() - t0) / steps
        assert nd == n
        # work counters (a separate counting call: window candidates from the level grids, candidate
        # pairs whose Hamming distance is computed, fixed-point passes) -> pairs per second of device
        # time; the VALU issue fraction of the search kernels comes from the committed PMC pass
        lib.orbfe_matcher_set_stats(1)
        m.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, th)
        lib.orbfe_matcher_set_stats(0)
        wst = (ctypes.c_longlong * 3)()
        lib.orbfe_matcher_last_stats(wst)
        mp = (matcher_pmc or {}).get(f"th{th}", {})
        # the search kernels: the PMC pass's names when it covers this th, else by the library's switch
        # (th < 4: k_sbp_multi0 + k_sbp_multi, the list-based passes; wider windows: k_sbp_band)
        kname = mp.get("kernel") or ("k_sbp_multi0+k_sbp_multi" if th < 4 else "k_sbp_band")
        out[f"th{th}"] = {"kernel": kname, "window_candidates": int(wst[0]), "pairs": int(wst[1]),
                          "passes": int(wst[2]), "pairs_per_s": round(wst[1] / (dms * 1e-3), 1),
                          "window_candidates_per_s": round(wst[0] / (dms * 1e-3), 1),
                          "valu_issue_frac": mp.get("valu_issue_frac"), "pmc_source": mp.get("source"),
                          "valu_per_pair": (round(mp["valu_per_call"] / max(int(wst[1]), 1), 2)
                                            if mp.get("valu_per_call") else None),"ms_per_call": round(dt * 1e3, 4), "calls_per_s": round(1.0 / dt, 2),
                          "queries_per_s": round(len(mps) / dt, 1), "device_ms_per_call": round(dms, 4),
                          "device_queries_per_s": round(len(mps) / (dms * 1e-3), 1),
                          "resident_ms_per_call": round(rdt * 1e3, 4),
                          "resident_queries_per_s": round(len(mps) / rdt, 1),
                          "resident_over_device": round(rdt * 1e3 / dms, 4),
                          "resident_wrapper_ms_per_call": round(wdt * 1e3, 4),
                          "resident_wrapper_over_device": round(wdt * 1e3 / dms, 4), "nmatches": int(n)}
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
                      "resident_ms_per_call: orbfe_search_by_projection_local_device wall time at the "
                      "C-ABI (ctypes, arguments prepared) with the records, slots and frame already in HBM; "
                      "resident_wrapper_ms_per_call: the same through the Python wrapper",
            "per_th": out}


def matcher_config5_n(steps, n_kp):
    """BASELINE config 5 at another frame size (N = 1000 and 5000): the same 100k-point
    local map construction (seed 12345) against an n_kp-keypoint frame, th in {1, 3, 5, 15}. Per th:
    the host C-ABI call (records packed + uploaded, slots back) and its device time (HIP events), and
    a parity check of the slots and count against the CPU oracle (outside the timed loop)."""
    from oracle import oracle
    from orb_slam3_ros_amd import synth_match as sm
    from orb_slam3_ros_amd.matcher import ORBmatcher
    oracle.build()
    rng = np.random.default_rng(12345)
    F = sm.synth_frame(rng, n_kp)
    mps = sm.synth_local_map(rng, F, 100_000)
    mvp0, obs = sm.initial_slots(rng, F.N)
    m = ORBmatcher(0.8)
    lib = m._lib
    out, all_ok = {}, True
    for th in (1, 3, 5, 15):
        a = mvp0.copy()
        n = m.SearchByProjectionLocalMap(F, a, obs, mps, th)
        b = mvp0.copy()
        no = oracle.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
        ok = n == no and np.array_equal(a, b)
        all_ok = all_ok and ok
        bufs = [mvp0.copy() for _ in range(steps)]
        t0 = time.perf_counter()
        for bb in bufs:
            m.SearchByProjectionLocalMap(F, bb, obs, mps, th)
        dt = (time.perf_counter() - t0) / steps
        lib.orbfe_matcher_set_timing(1)
        dev = []
        for _ in range(steps):
            m.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, th)
            dev.append(lib.orbfe_matcher_last_ms())
        lib.orbfe_matcher_set_timing(0)
        dms = float(np.mean(dev))
        out[f"th{th}"] = {"ms_per_call": round(dt * 1e3, 4), "device_ms_per_call": round(dms, 4),
                          "queries_per_s": round(len(mps) / dt, 1), "device_queries_per_s": round(len(mps) / (dms * 1e-3), 1),
                          "nmatches": int(n), "parity_ok": bool(ok)}
    return {"workload": f"SearchByProjection local map: 100k map points vs a {n_kp}-keypoint stereo frame "
                        "(BASELINE config 5's second frame size), nnratio 0.8, seed 12345",
            "per_th": out, "parity": {"ok": all_ok, "detail": "slots + nmatches identical to the CPU oracle per th"}}


def matcher_calls(steps):
    """The Tracking thread's other per-frame matcher calls at their own sizes, one host C-ABI call each
    through the Python wrapper (inputs packed and uploaded, results back), with the kernels' device
    time (HIP events), the CPU oracle's single-thread time on the same inputs and a parity check:
      - MonocularInitialization: ORBmatcher(0.9, true).SearchForInitialization(mInitialFrame,
        mCurrentFrame, mvbPrevMatched, mvIniMatches, 100) (Tracking.cc:2386) on 5000-feature frames
        (the initial extractor's 5 x nFeatures);
      - TrackReferenceKeyFrame: ORBmatcher(0.7, true).SearchByBoW(mpReferenceKF, mCurrentFrame)
        (Tracking.cc:2836);
      - Relocalization: ORBmatcher(0.75, true).SearchByBoW(pKF, mCurrentFrame) per candidate
        (Tracking.cc:3765), then ORBmatcher(0.9, true).SearchByProjection(mCurrentFrame, pKF, sFound,
        10, 100) (Tracking.cc:3818) and (..., 3, 64) (Tracking.cc:3838)."""
    from oracle import oracle
    from orb_slam3_ros_amd import synth_match as sm
    from orb_slam3_ros_amd.matcher import ORBmatcher
    oracle.build()
    lib = ORBmatcher()._lib
    rng = np.random.default_rng(4242)

    def timed(gpu_call, cpu_call, check):
        gpu_call()   # warm-up (buffers, grids)
        t, dev = [], []
        lib.orbfe_matcher_set_timing(1)
        for _ in range(steps):
            t0 = time.perf_counter()
            g = gpu_call()
            t.append(time.perf_counter() - t0)
            dev.append(lib.orbfe_matcher_last_ms())
        lib.orbfe_matcher_set_timing(0)
        tc = []
        for _ in range(max(3, min(steps, 10))):
            t0 = time.perf_counter()
            c = cpu_call()
            tc.append(time.perf_counter() - t0)
        ms, cms = 1e3 * float(np.median(t)), 1e3 * float(np.median(tc))
        return {"ms_per_call": round(ms, 4), "device_ms_per_call": round(float(np.median(dev)), 4),
                "cpu_ms_per_call": round(cms, 4), "speedup_vs_cpu": round(cms / ms, 2),
                "parity_ok": bool(check(g, c))}

    out = {}
    # monocular initialisation, 5000 features, window 100
    F1 = sm.synth_frame(rng, 5000, stereo=False)
    F2, _ = sm.perturbed_frame(rng, F1, shift=(6.0, -4.0), jitter=2.0, rot=12.0, flip_p=0.06, drop=0.2)
    prev0 = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)

    def sfi(m):
        pv, m12 = prev0.copy(), np.zeros(F1.N, np.int32)
        return m.SearchForInitialization(F1, F2, pv, m12, 100), pv, m12
    og, oo = ORBmatcher(0.9, True), oracle.OracleMatcher(0.9, True)
    out["search_for_initialization_5000"] = dict(
        timed(lambda: sfi(og), lambda: (lambda pv, m12: (oo.search_for_init(F1, F2, pv, m12, 100), pv, m12))(
            prev0.copy(), np.zeros(F1.N, np.int32)),
              lambda g, c: g[0] == c[0] and np.array_equal(g[1], c[1]) and np.array_equal(g[2], c[2])),
        features=int(F1.N), window=100)
    # SearchByBoW(KF, F): reference keyframe (0.7) and relocalisation candidate (0.75), 1000 features
    KF = sm.synth_frame(rng, 1000, stereo=False)
    F, src = sm.perturbed_frame(rng, KF, rot=20.0, flip_p=0.05, drop=0.15)
    kf_mp = np.where(rng.random(KF.N) < 0.25, -1, np.arange(KF.N) + 100).astype(np.int32)
    fk, ff = sm.synth_bow(rng, 400, KF, F, src)
    for name, ratio in (("search_by_bow_track_reference_kf", 0.7), ("search_by_bow_relocalisation", 0.75)):
        g_m, o_m = ORBmatcher(ratio, True), oracle.OracleMatcher(ratio, True)
        out[name] = dict(timed(lambda: g_m.SearchByBoW(KF.keys, KF.desc, kf_mp, fk, F, ff),
                               lambda: o_m.search_by_bow(KF.keys, KF.desc, kf_mp, fk, F, ff),
                               lambda g, c: g[0] == c[0] and np.array_equal(g[1], c[1])),
                         kf_features=int(KF.N), frame_features=int(F.N), bow_nodes=400)
    # relocalisation's SearchByProjection(F, KF, sFound, th, ORBdist): the candidate keyframe's points
    Fr = sm.synth_frame(rng, 1000, stereo=False)
    pts = sm.synth_proj_points(rng, Fr, 1200, copy_frac=0.7)
    mvp0, _ = sm.initial_slots(rng, Fr.N, 0.25)
    g_m, o_m = ORBmatcher(0.9, True), oracle.OracleMatcher(0.9, True)
    for th, orbdist in ((10, 100), (3, 64)):
        def gk():
            a = mvp0.copy()
            return g_m.SearchByProjectionKeyFrame(Fr, a, pts, th, orbdist), a

        def ck():
            b = mvp0.copy()
            return o_m.sbp_kf(Fr, b, pts, th, orbdist), b
        out[f"search_by_projection_keyframe_th{th}"] = dict(
            timed(gk, ck, lambda g, c: g[0] == c[0] and np.array_equal(g[1], c[1])),
            frame_features=int(Fr.N), kf_points=int(len(pts)), ORBdist=orbdist)
    return {"workload": "synthetic Tracking-sized inputs, seed 4242 (sm.synth_frame / perturbed_frame / synth_bow / "
                        "synth_proj_points)",
            "timing": "median over the calls: ms_per_call = the wrapper's host C-ABI call (inputs packed and "
                      "uploaded, results back); device_ms_per_call = its kernels (HIP events); cpu_ms_per_call = the "
                      "oracle restatement on one host thread, same inputs",
            "calls": out, "parity": {"ok": all(v["parity_ok"] for v in out.values()),
                                     "detail": "counts and outputs identical to the CPU oracle per call"}}


def make_images(rank, W, H, F, U, dev, seed0=0):
    """Interleaved [2F, H, W] device tensor of U distinct synthetic stereo pairs tiled over F frames
    (frame f = pair f % U); returns (images, host pairs, frame -> pair map)."""
    import torch
    from orb_slam3_ros_amd.synth import synth_stereo
    U = min(U, F)
    pairs = [synth_stereo(seed0 + 1000 * rank + i, W, H) for i in range(U)]
    host = np.empty((2 * F, H, W), np.uint8)
    for f in range(F):
        host[2 * f], host[2 * f + 1] = pairs[f % U]
    return torch.from_numpy(host).to(dev), pairs, np.arange(F) % U


def time_steps(fe, images, steps, warmup):
    import torch
    for _ in range(warmup):
        fe.run(images)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fe.run(images)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def stage_times(fe, images, n):
    import torch
    fe.set_stage_timing(True)
    for _ in range(n):
        fe.run(images)
    torch.cuda.synchronize()
    st, _ = fe.stage_timing()
    fe.set_stage_timing(False)
    return st


def pmc_valu(n_img, w, h):
    """Per-kernel VALU instruction counts and wave states from the newest committed PMC summary of
    this workload (profiles/rNN_pmc_valu.json, tools/pmc_round.py)."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_valu.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("images_per_step"), d.get("width"), d.get("height")) == (n_img, w, h):
            best = (d["kernels"], os.path.basename(f))
    return best


def write_sequence_job(path, frames, W=752, H=480, nf=1000, window=20, seed=21, cxy=None):
    """The drop-in harness's input (tests/native/capi_frontend.cpp SeqJob): a seeded synthetic stereo
    sequence (synth.synth_stereo_sequence: a planar scene at disparity SEQ_DISP, the rig moving SEQ_SHIFT
    px per frame, every frame distinct) with the EuRoC MH_01 pinhole intrinsics and the per-frame
    translation that makes the constant-velocity motion model exact."""
    import struct
    from orb_slam3_ros_amd.synth import SEQ_DISP, SEQ_SHIFT, synth_stereo_sequence
    fx, fy, cx, cy = EUROC_FX, 457.296, 367.215, 248.375
    if cxy is not None:   # a principal point for another image size (the 512x512 two-camera rig)
        cx, cy = float(cxy[0]), float(cxy[1])
    bf = EUROC_BF
    tx = SEQ_SHIFT * (bf / SEQ_DISP) / fx
    seq = synth_stereo_sequence(seed, frames, W, H)
    with open(path, "wb") as f:
        f.write(struct.pack("<6i6f", 0x5342524F, W, H, nf, frames, window, fx, fy, cx, cy, bf, tx))
        for left, right in seq:
            f.write(left.tobytes())
            f.write(right.tobytes())
    return path


def dropin_leg(frames, W=752, H=480, nf=1000, tracking_frames=60, cpu=True):
    """The drop-in path at batch 1 (rank 0, not part of `value`), timed by the compiled C++ consumer of
    the C-ABI (tests/native/capi_frontend.cpp, linked against liborbfe.so only) over a seeded synthetic
    stereo SEQUENCE (every frame a distinct pair, small per-frame shifts), host images in and host
    results out:
      frame_call: orbfe_frame_stereo, Frame::Frame(stereo) in one call (Frame.cc:101-141);
      threads:    two ORBextractor::operator() calls on two per-frame std::threads, then
                  ComputeStereoMatches (Frame.cc:122-141), the way the reference builds the Frame;
      tracking:   a whole Tracking frame (tests/native/tracking_loop.h): Frame(stereo), then
                  SearchByProjection(CurrentFrame, LastFrame, th 7) (Tracking.cc:2925) and
                  SearchLocalPoints (isInFrustum + SearchByProjection(F, local map, th 1),
                  Tracking.cc:3382-3452), with the same loop run on the CPU restatement beside it
                  (tests/native/tracking_cpu.cpp) and the two runs' per-frame results compared.
    frame_ms = median wall time per frame without event timing; split_ms from a second, timed pass."""
    import subprocess
    import tempfile
    from orb_slam3_ros_amd import build as B
    binary = B.CAPI_BIN
    if not os.path.exists(binary):
        return {"error": "tests/native/capi_frontend not built (run __graft_entry__.build())"}
    n_seq = max(frames, tracking_frames)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        job = write_sequence_job(os.path.join(d, "seq.bin"), n_seq, W, H, nf)
        r = subprocess.run([binary, "--latency", str(frames), job], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            return {"error": (r.stderr or r.stdout)[-400:]}
        lat = json.loads(r.stdout.strip().splitlines()[-1])
        out.update(lat["frame_call"])
        out["threads"] = lat["threads"]
        out["frames"], out["distinct_pairs"] = lat["frames"], lat["distinct_pairs"]
        out["path"] = ("host C-ABI per frame over a seeded stereo sequence: orbfe_frame_stereo (Frame(stereo) in one "
                       "call: one upload, one two-image launch chain with the stereo kernels, one result copy); "
                       "`threads` = orbfe_extract L || R on two std::threads + orbfe_stereo_match")
        if tracking_frames > 0:
            g_out, c_out = os.path.join(d, "gpu.out"), os.path.join(d, "cpu.out")
            r = subprocess.run([binary, "--tracking", str(tracking_frames), job, g_out], capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                out["tracking"] = {"error": (r.stderr or r.stdout)[-400:]}
            else:
                tr = json.loads(r.stdout.strip().splitlines()[-1])
                if cpu and os.path.exists(B.TRACK_CPU_BIN):
                    # CHECKER + CPU baseline: the same loop on the oracle restatement
                    rc = subprocess.run([B.TRACK_CPU_BIN, str(tracking_frames), job, c_out], capture_output=True,
                                        text=True, timeout=600)
                    if rc.returncode == 0:
                        tc = json.loads(rc.stdout.strip().splitlines()[-1])
                        same = open(g_out, "rb").read() == open(c_out, "rb").read()
                        tr["cpu"] = {"tracking_frame_ms": tc["tracking_frame_ms"], "split_ms": tc["split_ms"],
                                     "path": tc["path"]}
                        tr["speedup_vs_cpu"] = round(tc["tracking_frame_ms"] / tr["tracking_frame_ms"], 2)
                        tr["parity"] = ("every frame's counts and mvpMapPoints identical to the CPU restatement's run"
                                        if same else "MISMATCH against the CPU restatement's run")
                        tr["parity_ok"] = same
                    else:
                        tr["cpu"] = {"error": (rc.stderr or rc.stdout)[-400:]}
                out["tracking"] = tr
                out["tracking_frame_ms"] = tr["tracking_frame_ms"]
            # BASELINE config 4 per frame: the KannalaBrandt8 two-camera Tracking frame (tests/native/
            # tracking_kb8.h) over a 512x512 sequence, with the CPU restatement beside it as checker
            kjob = write_sequence_job(os.path.join(d, "seq_kb8.bin"), tracking_frames, 512, 512, nf, 20, 31,
                                      (256.0, 256.0))
            gk, ck = os.path.join(d, "gpu_kb8.out"), os.path.join(d, "cpu_kb8.out")
            r = subprocess.run([binary, "--tracking-kb8", str(tracking_frames), kjob, gk], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                out["tracking_kb8"] = {"error": (r.stderr or r.stdout)[-400:]}
            else:
                tk = json.loads(r.stdout.strip().splitlines()[-1])
                if cpu and os.path.exists(B.TRACK_CPU_BIN):
                    rc = subprocess.run([B.TRACK_CPU_BIN, "--kb8", str(tracking_frames), kjob, ck], capture_output=True,
                                        text=True, timeout=600)
                    if rc.returncode == 0:
                        tc = json.loads(rc.stdout.strip().splitlines()[-1])
                        same = open(gk, "rb").read() == open(ck, "rb").read()
                        tk["cpu"] = {"tracking_frame_ms": tc["tracking_frame_ms"], "split_ms": tc["split_ms"],
                                     "path": tc["path"]}
                        tk["speedup_vs_cpu"] = round(tc["tracking_frame_ms"] / tk["tracking_frame_ms"], 2)
                        tk["parity_ok"] = same
                        tk["parity"] = ("every frame's counts and both cameras' mvpMapPoints identical to the CPU "
                                        "restatement's run" if same else "MISMATCH against the CPU restatement's run")
                    else:
                        tk["cpu"] = {"error": (rc.stderr or rc.stdout)[-400:]}
                out["tracking_kb8"] = tk
    return out


def config4_dist_leg(dev, rank, world, gloo, K=64, steps=10, warmup=3):
    """BASELINE config 4's own multi-GPU layout (world even, every rank): 512x512 KannalaBrandt8-like
    stereo, stream s's left / right camera on ranks 2s / 2s + 1 (distributed.rig_role), K frames of
    the rank's camera extracted per step (vLappingArea {0, 511}), one slab all-gather per step (K
    steps batched per collective), the fisheye kNN + ratio of the step's K frames on
    the left rank against the partner's gathered slots, one step behind so the gather overlaps the
    next extraction. Frames/s = streams x K x steps / max-rank time. The left ranks' last step is
    checked against the CPU oracle afterwards (4 frames). With K = 1, ms_per_step is the per-frame
    step time of the rig (a frame's kNN completes one step after its extraction)."""
    import torch
    import torch.distributed as dist
    from orb_slam3_ros_amd import distributed as odist
    from orb_slam3_ros_amd.synth import synth_stereo
    stream, cam = odist.rig_role(rank)
    U = 8   # distinct synthetic pairs per stream, tiled over the K frames
    rig, err = None, None
    try:
        pairs = [synth_stereo(31000 + 100 * stream + i, 512, 512) for i in range(U)]
        imgs = torch.from_numpy(np.stack([pairs[f % U][cam] for f in range(K)])).to(dev)
        rig = odist.StereoRigExchange(K, 512, 512, device=dev)
    except Exception as e:  # noqa: BLE001 - every rank learns of it below, so none waits in a collective
        err = f"{type(e).__name__}: {e}"[:400]
    ready = torch.tensor([0 if err else 1], dtype=torch.int32, device="cpu" if gloo else dev)
    dist.all_reduce(ready, op=dist.ReduceOp.MIN)
    if not int(ready.item()):
        if rig is not None:
            rig.close()
        return {"error": err or "set-up failed on another rank"}
    it = [0]

    def step():
        k = it[0]
        it[0] += 1
        rig.extract(imgs, k)
        if k:
            rig.match(k - 1)

    def finish():
        rig.match(it[0] - 1)
        rig.drain()

    # Every rank reaches the same collectives in the same order whatever fails locally:
    # a rank whose loop or checker raises records the error, skips only local work, and still joins
    # the barrier / all_reduce(el) / all_reduce(flag) below. A failure INSIDE a step's own all-gather
    # cannot be bridged this way; the process group's timeout (init in main) ends that case.
    err = None
    t0 = time.perf_counter()
    try:
        for _ in range(warmup):
            step()
        finish()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - reported in the leg's result
        err = f"warmup: {type(e).__name__}: {e}"[:400]
    dist.barrier()
    if err is None:
        t0 = time.perf_counter()
        try:
            for _ in range(steps):
                step()
            finish()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            err = f"timed loop: {type(e).__name__}: {e}"[:400]
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cpu" if gloo else dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    ok, detail = err is None, err or "right-camera rank (no kNN)"
    try:
        if cam == 0 and err is None:   # CHECKER, outside the timed region
            from oracle import oracle
            oracle.build()
            l2r = rig.l2r.cpu().numpy()
            ngood = rig.ngood.cpu().numpy()
            for f in range(min(4, K)):
                left, right = pairs[f % U]
                ol, orr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
                ml, kl, dl = ol(left, (0, 511))
                mr, kr, dr = orr(right, (0, 511))
                g, t, _ = oracle.stereo_knn_ratio(dl[ml:], dr[mr:], 0.7)
                exp = np.full(rig.cap, -1, np.int32)
                exp[ml:len(kl)][t >= 0] = t[t >= 0] + mr
                if int(ngood[f]) != g or not np.array_equal(l2r[f], exp):
                    ok, detail = False, f"stream {stream} frame {f}: kNN candidates differ from the oracle"
                    break
            else:
                detail = f"stream {stream}: frames 0..3 of the last step bit-exact vs the CPU oracle"
    except Exception as e:  # noqa: BLE001
        ok, detail = False, f"checker: {type(e).__name__}: {e}"[:400]
    finally:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cpu" if gloo else dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    rig.close()
    streams = world // 2
    return {"workload": "TUM-VI-like 512x512 KannalaBrandt8 stereo (BASELINE config 4): one camera per rank, "
                        f"{streams} stream(s) x 2 cameras, K={K} frames per step and collective, vLappingArea "
                        "{0,511}, slot all-gather + batched knnMatch(k=2)+ratio on the left-camera rank",
            "frames_per_s": round(streams * K * steps / el, 2), "images_per_s": round(world * K * steps / el, 2),
            "ms_per_step": round(1000.0 * el / steps, 4), "steps": steps, "warmup": warmup, "K": K,
            "allgather_bytes_per_rank_per_step": odist.slab_bytes(K, rig.cap), "backend": "gloo" if gloo else "nccl",
            "parity": {"ok": bool(int(flag.item())), "detail_rank0": detail}}


def side_leg(dev, name, W, H, nf, F, steps, warmup, stereo, lap, bf, fx, check_frames, seed0):
    """A secondary BASELINE config on this GPU (rank 0, not part of `value`): throughput, stage
    times, the pyramid+FAST kernel roofline and a post-timing parity check."""
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    images, pairs, fmap = make_images(0, W, H, F, 8, dev, seed0)
    fe = StereoFrontEnd(F, W, H, nfeatures=nf, bf=bf, fx=fx, device=dev, lap_left=lap, lap_right=lap, stereo=stereo)
    sec = time_steps(fe, images, steps, warmup)
    st = stage_times(fe, images, max(3, steps // 2))
    pf = st["pyramid_fast"]
    nb = algorithmic_bytes(W, H)
    ok, msg = parity_check(fe, pairs, fmap, min(check_frames or F, F), nf, bf, fx, stereo=stereo, lap=lap)
    out = {"workload": name, "frames_per_step": F, "images_per_step": 2 * F, "ms_per_step": round(sec * 1e3, 4),
           "frames_per_s": round(F / sec, 2), "stage_ms": {k: round(v, 4) for k, v in st.items()},
           "pyramid_fast_roofline": {"achieved_GBps": round(2 * F * nb / (pf * 1e-3) / 1e9, 1),
                                     "frac": round(2 * F * nb / (pf * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "bytes_per_image": nb, "kernel_ms_per_launch": round(pf, 4)},
           "stereo_matches_per_frame_mean": float(fe.nmatch.float().mean().item()),
           "parity": {"ok": ok, "detail": msg}}
    fe.close()
    return out, ok


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(argv, gpus, port, python=sys.executable, script=None):
    """The torchrun command line that runs this bench as `gpus` ranks on one node (one process per
    GPU, rendezvous on 127.0.0.1), forwarding argv unchanged so every rank parses the same flags."""
    return [python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)


def maybe_launch(gpus, argv, env=None):
    """`bench.py --gpus N` without an outer torchrun: spawn N ranks as a CHILD process (never exec:
    nothing here has touched the GPU yet, and the parent never will) and return its exit code, the
    rank-0 JSON line reaching our stdout through the inherited descriptor. Returns None when this
    process is itself a rank (WORLD_SIZE set, equal to --gpus) or N = 1. A WORLD_SIZE that disagrees
    with --gpus is an error: the line must never report fewer GPUs than were asked for."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}", file=sys.stderr, flush=True)
            return 2
        return None
    if gpus <= 1:
        return None
    child_env = dict(env)
    child_env.setdefault("MASTER_ADDR", "127.0.0.1")
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(launch_command(argv, gpus, _free_port()), env=child_env)
    return r.returncode


def launch_dry_run(args):
    """--launch-dry-run: the rank plumbing alone (no GPU call): every rank joins a gloo group,
    all-reduces its rank, and rank 0 prints the line's n_gpus. The CPU test of maybe_launch."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "rank_sum": int(t.item()), "gpus_flag": args.gpus, "dry_run": True}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=512, help="stereo frames per GPU per step (512: 1024 images per launch, +3 %% over 256, tools/gpu_frames_sweep.sh)")
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--unique", type=int, default=32, help="distinct synthetic frames (tiled over the batch)")
    ap.add_argument("--pipelines", type=int, default=1, help="sub-batches on separate HIP streams")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the post-timing oracle check (profiling runs)")
    ap.add_argument("--parity-frames", type=int, default=0, help="frames checked after timing (0: the whole batch)")
    ap.add_argument("--no-side-configs", action="store_true", help="skip the config 3 / config 4 legs")
    ap.add_argument("--stage-steps", type=int, default=10, help="extra steps with per-stage HIP events")
    ap.add_argument("--matcher-steps", type=int, default=50, help="config-5 SearchByProjection calls per th (0: skip)")
    ap.add_argument("--dropin-frames", type=int, default=100, help="batch-1 drop-in latency frames (0: skip)")
    ap.add_argument("--rectify-steps", type=int, default=5,
                    help="time cv::remap rectification of the step's images (reported separately; 0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the measured path); gloo = CPU rehearsal of the multi-rank path")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses cuda:0 (rehearse N ranks on a 1-GPU box with --dist-backend gloo)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="only the rank plumbing of --gpus N (gloo, no GPU): rank 0 prints n_gpus")
    args = ap.parse_args()

    rc = maybe_launch(args.gpus, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.launch_dry_run:
        launch_dry_run(args)
        return

    native = (None, None)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        native = start_native_oracle_build()   # compiles while the GPU legs run

    import torch
    import torch.distributed as dist
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    from orb_slam3_ros_amd import distributed as odist

    local_rank = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gloo:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=300))

    W, H, F = args.width, args.height, args.frames
    bf, fx = EUROC_BF, EUROC_FX
    images, pairs, fmap = make_images(rank, W, H, F, args.unique, dev)
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

    # ---- checker: the last timed step's outputs against the CPU oracle (outside the timed region)
    parity = None
    if not args.no_parity:
        ok, msg = parity_check(fe, pairs, fmap, min(args.parity_frames or F, F), args.nfeatures, bf, fx)
        parity = {"ok": ok, "detail": msg, "rank": rank}
        if not ok:
            print(json.dumps({"parity": parity}), file=sys.stderr, flush=True)
            sys.exit(3)

    # per-stage HIP-event timing on the launch stream (separate steps, same workload, one pipeline
    # so the events bracket kernels that run alone on the GPU)
    fe_t = fe if args.pipelines == 1 else StereoFrontEnd(F, W, H, nfeatures=args.nfeatures, bf=bf, fx=fx, device=dev)
    stages = stage_times(fe_t, images, args.stage_steps)
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
        rbytes = images.numel() * (1 + 1) + 2 * 4 * W * H   # read + write per image, maps once
        rect = {"ms_per_step": round(rms, 4), "images": int(images.shape[0]),
                "achieved_GBps": round(rbytes / (rms * 1e-3) / 1e9, 1),
                "algorithmic_bytes_per_step": int(rbytes)}
        del rout
    counts = fe.counts.cpu().numpy()
    nm = fe.nmatch.cpu().numpy()
    c4 = c4k1 = None
    if world > 1 and world % 2 == 0 and not args.no_side_configs:
        # config 4's own layout over the same ranks (after the config-2 measurement, not part of `value`):
        # K = 64 frames per collective (throughput), then K = 1 (one frame per step and all-gather: the
        # per-frame cadence a live rig runs at)
        try:
            c4 = config4_dist_leg(dev, rank, world, gloo)
        except Exception as e:  # noqa: BLE001 - reported, never fatal to the config-2 line
            c4 = {"error": f"{type(e).__name__}: {e}"[:400]}
        try:
            c4k1 = config4_dist_leg(dev, rank, world, gloo, K=1, steps=60, warmup=5)
        except Exception as e:  # noqa: BLE001
            c4k1 = {"error": f"{type(e).__name__}: {e}"[:400]}

    if rank == 0:
        n_img = 2 * F
        pyr_fast_ms = stages["pyramid_fast"]
        pf_kernel = "pyramid+FAST pass: k_resize_s x7 + k_fast"
        bytes_img = algorithmic_bytes(W, H)
        achieved = n_img * bytes_img / (pyr_fast_ms * 1e-3) / 1e9 if pyr_fast_ms > 0 else 0.0
        dominant = max(stages, key=stages.get)
        tr = pmc_traffic(n_img, W, H)
        cache = pmc_cache(n_img, W, H)
        valu = pmc_valu(n_img, W, H)
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
                "kernel": pf_kernel,
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
            "parity": parity,
        }
        if valu is not None:
            # VALU issue fraction per kernel (committed rocprofv3 counters of this workload on the
            # isolated-timing build: SQ_INSTS_VALU per step over the kernel's own trace time x the
            # wave64 issue peak, 1024 SIMD-32s x 2.4 GHz / 2 cycles), and for the pyramid+FAST pass as
            # timed in this run
            vk = valu[0]
            # the pyramid kernels: k_resize_s (row-streamed, the default) and / or k_resize (LDS-tiled)
            pyr_k = [k for k in vk if k.startswith("k_resize")]
            result["roofline"]["valu_issue_frac"] = {k: v["valu_issue_frac"] for k, v in vk.items()
                                                     if k in pyr_k or k in ("k_fast", "k_octree", "k_describe",
                                                                            "k_stereo")}
            if pyr_k and "k_fast" in vk and pyr_fast_ms > 0:
                result["roofline"]["valu_issue_frac_pass"] = round(
                    (sum(vk[k]["valu_per_step"] for k in pyr_k) + vk["k_fast"]["valu_per_step"])
                    / (pyr_fast_ms * 1e-3) / VALU_ISSUE_PEAK, 4)
            result["roofline"]["wave_states"] = {k: vk[k]["wave_state"] for k in pyr_k + ["k_fast"] if k in vk}
            result["roofline"]["valu_source"] = valu[1]
        if cache is not None and "k_describe" in cache[0]:
            kd = cache[0]["k_describe"]
            result["describe_pass"] = {"kernel": "k_describe", "l2_hit_rate": kd["l2_hit_rate"],
                                       "lds_bank_conflict_share": kd["lds_conflict_share"], "source": cache[1]}
        if rect is not None:
            if tr is not None and "k_remap" in tr_kernels(n_img, W, H):
                rk = tr_kernels(n_img, W, H)["k_remap"]
                rect["pmc_traffic_bytes_per_step"] = rk["read_bytes_per_step"] + rk["write_bytes_per_step"]
            result["rectify_remap"] = rect
        if c4 is not None:
            result["config4_multi_gpu"] = c4
        if c4k1 is not None:
            result["config4_multi_gpu_k1"] = c4k1
        if world == 1 and not args.no_side_configs:
            legs, all_ok = {}, True
            legs["config3"], ok3 = side_leg(dev, "KITTI-like stereo 1241x376, nFeatures 2000 (BASELINE config 3): "
                                                 "extract L+R + ComputeStereoMatches", 1241, 376, 2000, 256,
                                            max(3, args.steps // 2), 2, "rectified", (0, 0), KITTI_BF, KITTI_FX, 0,
                                            20000)
            legs["config4_step"], ok4 = side_leg(dev, "TUM-VI-like 512x512 KannalaBrandt8 stereo: the whole "
                                                      "BASELINE config 4 step (4 synthetic streams x 2 cameras = 8 "
                                                      "images) on ONE GPU (config 4 spreads it over 8 GPUs, one "
                                                      "image each), vLappingArea {0,511}, batched "
                                                      "knnMatch(k=2)+ratio", 512, 512, 1000, 4,
                                                 max(10, args.steps), 3, "fisheye", (0, 511), 0.0, 1.0, 0, 21000)
            legs["config4_batch"], ok4b = side_leg(dev, "as config4_step at a 512-image batch (throughput)", 512, 512,
                                                   1000, 256, max(3, args.steps // 2), 2, "fisheye", (0, 511), 0.0,
                                                   1.0, 0, 22000)
            legs["config2_nf1200"], ok2b = side_leg(dev, "EuRoC-like stereo 752x480, nFeatures 1200 (config/Stereo/"
                                                         "EuRoC.yaml; BASELINE config 2's secondary size): extract L+R "
                                                         "+ ComputeStereoMatches", 752, 480, 1200, 512,
                                                    max(3, args.steps // 2), 2, "rectified", (0, 0), EUROC_BF, EUROC_FX,
                                                    0, 23000)
            result["side_configs"] = legs
            if not (ok3 and ok4 and ok4b and ok2b):
                print(json.dumps(result), file=sys.stderr, flush=True)
                sys.exit(3)
        if args.matcher_steps > 0:
            result["matcher_config5"] = matcher_config5(args.matcher_steps)
            if world == 1 and not args.no_side_configs:
                c5b = matcher_config5_n(max(5, args.matcher_steps // 5), 5000)
                result["matcher_config5_n5000"] = c5b
                mc = matcher_calls(max(10, args.matcher_steps // 2))
                result["matcher_calls"] = mc
                if not (c5b["parity"]["ok"] and mc["parity"]["ok"]):
                    print(json.dumps(result), file=sys.stderr, flush=True)
                    sys.exit(3)
        if args.dropin_frames > 0 and world == 1:
            dl = dropin_leg(args.dropin_frames, nf=args.nfeatures, cpu=not args.no_cpu_baseline)
            result["dropin"] = dl
            result["dropin_latency_ms"] = dl.get("frame_ms")
        if not args.no_cpu_baseline and world == 1:
            result["cpu_baseline"] = cpu_baseline(native)
            lr2t = result["cpu_baseline"].get("latency_lr2t")
            if result.get("dropin_latency_ms") and lr2t:
                result["dropin"]["cpu_latency_lr2t_ms"] = lr2t
                result["dropin"]["speedup_vs_cpu_latency_lr2t"] = round(lr2t / result["dropin_latency_ms"], 2)
        print(json.dumps(result), flush=True)
    fe.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

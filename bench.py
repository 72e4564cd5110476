#!/usr/bin/env python3
"""Benchmark: Mrays/s + frame time of the MI355X render path on BASELINE.json's workload.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ultracomplex_1080p64|...]

A step = one frame, timed as SURVEY.md §8(d) / BASELINE.md §3 define it: from the render launch until the frame's
Color[W*H] is in host memory (the buffer main.c:305 hands to stbi_write_bmp).  Rank r of N renders the interleaved
rows y = r + k*N (main.c:84 lifted to GPUs) with the HIP kernels and copies them with its own SDMA engines straight
into their places of the shared host frame (rtc_frame_loop: native pipelined frames, rtc_copy_rows_d2h_dma; a POSIX
shared-memory frame every rank maps at N > 1) -- the reference's threads likewise write their rows into one image
(main.c:285-302).  At N > 1 the RCCL path is measured beside it: the parts gathered to rank 0's GPU over xGMI
(torch.distributed `nccl` = RCCL) and re-interleaved there (the device-resident frame).  The scene (the reference
loader's Triangle[], tests/golden/scenes) is resident in HBM before timing.

Prints ONE JSON line on rank 0.  `value` = W*H*spp*K / t / 1e6 over the whole job (strong scaling: the frame is
fixed, N GPUs split it).  `roofline` covers the split launch's kernels (rtc_render_chain, rtc_render_sky) with the
live HIP-event times and the committed rocprofv3 PMC digest of the same workload (profiles/); `cpu_baseline` is the
CPU restatement of the reference (oracle/, "port") on the box's host cores beside the reference itself compiled here
(oracle/_ref/rtc_ref), rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import queue
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mrays/sec + frame time, 1920x1080x64spp ultracomplex.obj, 1/2/4/8 GPUs"
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (FP32 vector, spec)
HBM_PEAK_GBS = 8000.0
FLOPS_PER_TEST = 57  # full rayTriangle path
# BASELINE.json configs: C1 simplest 256x256x1 (CPU), C2 cube 1080p16, C3 fsuzane 1080p64, C4 complex 4K64,
# C5 ultracomplex 4K256, NS ultracomplex 4K64; the metric's own config is ultracomplex 1080p64
WORKLOADS = {
    "ultracomplex_1080p64": ("ultracomplex", 1920, 1080, 64),
    "ultracomplex_4k64": ("ultracomplex", 3840, 2160, 64),
    "ultracomplex_4k256": ("ultracomplex", 3840, 2160, 256),
    "complex_4k64": ("complex", 3840, 2160, 64),
    "fsuzane_1080p64": ("fsuzane", 1920, 1080, 64),
    "cube_1080p16": ("cube", 1920, 1080, 16),
    "simplest_256p1": ("simplest", 256, 256, 1),
}
REF_THREADS = 12  # main.c:43 NUMBER_OF_THREADS


def load_scene(name):
    import numpy as np

    from raytracingc_amd import TRIANGLE_DT

    raw = open(os.path.join(REPO, "tests", "golden", "scenes", name + ".tris"), "rb").read()
    count, tonly = np.frombuffer(raw[:8], np.int32)
    return np.frombuffer(raw[8:8 + 68 * int(count)], TRIANGLE_DT).copy(), int(tonly)


# ---- CPU baseline --------------------------------------------------------------------------------------
def cpu_info() -> dict:
    """lscpu model and topology, nproc, and this process's CPU share (affinity, cgroup quota)."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name", "")
        info["sockets"] = int(kv.get("Socket(s)", "0") or 0)
        info["cores_per_socket"] = int(kv.get("Core(s) per socket", "0") or 0)
        info["threads_per_core"] = int(kv.get("Thread(s) per core", "0") or 0)
    except Exception:
        pass
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpus"] = None if q == "max" else round(int(q) / int(p), 2)
    except Exception:
        info["cgroup_cpus"] = None
    return info


def cpu_baseline(tris, tonly, scene, cam, W, H, spp, budget_samples, gpu_colors, gpu_accum):
    """The reference algorithm on the host: the CPU restatement (oracle/rtc_oracle.c, bit-identical to the
    reference on every golden fixture; gcc -O3, no FMA) with row-interleaved pthreads like main.c:84, at the
    threads this process may actually run (min(nproc, affinity, cgroup quota)), at nproc and at the reference's 12;
    `value` is the fastest of them.  The reference's own sources compiled here (oracle/_ref/rtc_ref, 12 threads,
    its own main) are timed beside it when the whole frame fits the budget.  Rows y = 0, s, 2s, ... of the same
    frame with s = ceil(samples / budget) (s = 1 at the metric's config)."""
    import hashlib

    import numpy as np

    import oracle.binding as orc
    import raytracingc_amd as rt
    from raytracingc_amd._abi import RtcRenderDesc

    info = cpu_info()
    stride = max(1, math.ceil(W * H * spp / budget_samples))
    d = RtcRenderDesc(W, H, spp, 10, tonly, 0, stride, 0)

    def run(threads):
        t0 = time.perf_counter()
        colors, accum, seg = orc.render(tris, None, scene, cam, d, threads=threads)
        return time.perf_counter() - t0, colors, accum, seg

    n_all = info["nproc"]
    quota = info.get("cgroup_cpus")
    usable = min(n_all, info.get("affinity", n_all), int(quota) if quota else n_all)
    counts = sorted({max(1, usable), n_all, REF_THREADS})
    runs = {}
    ccol = cacc = seg = None
    for n in counts:
        dt, col, acc, sg = run(n)
        runs[n] = dt
        if ccol is None:
            ccol, cacc, seg = col, acc, sg
    rows = ccol.shape[0]
    samples = rows * W * spp
    best = min(runs, key=runs.get)
    res = {
        "value": round(samples / runs[best] / 1e6, 3), "unit": "Mrays/s", "cores": best, "kind": "port",
        "threads": best,
        "by_threads": {str(n): round(samples / t / 1e6, 3) for n, t in sorted(runs.items())},
        "usable_cpus": usable,
        "cpu_model": info.get("model"),
        "topology": f"{info.get('sockets')} sockets x {info.get('cores_per_socket')} cores x "
                    f"{info.get('threads_per_core')} SMT = nproc {info['nproc']}; affinity {info['affinity']} CPUs, "
                    f"cgroup quota {info.get('cgroup_cpus')} CPUs",
        "sample": (f"{'the whole frame' if stride == 1 else f'rows y = 0 mod {stride} of the frame'} ({rows} rows x "
                   f"{W} x {spp} spp = {samples} samples, {seg} segments), render loop only, timed at "
                   + ", ".join(f"{n} threads {runs[n]:.2f} s" for n in counts)
                   + "; value = the fastest; oracle/rtc_oracle.c (gcc -O3, no FMA)"),
    }
    g_rows = gpu_colors[::stride]
    res["u8_mismatch_vs_gpu"] = int((g_rows != ccol).any(-1).sum())
    res["float_bits_equal_vs_gpu"] = bool(gpu_accum is not None and
                                          np.array_equal(gpu_accum[::stride].view(np.uint32), cacc.view(np.uint32)))
    ref_bin = orc.REF_BIN
    if os.path.exists(ref_bin) and W * H * spp <= 1.5 * budget_samples:
        with tempfile.TemporaryDirectory() as tmp:
            obj = os.path.join(tmp, "scene.obj")
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from obj_export import write_obj  # the fixture as an OBJ + MTL the reference loads byte for byte

            write_obj(obj, tris)
            bmp = os.path.join(tmp, "ref.bmp")
            t0 = time.perf_counter()
            r = subprocess.run([ref_bin, "--spp", str(spp), "-i", obj, "-s", str(W), str(H), "-o", bmp], cwd=tmp,
                               capture_output=True, text=True, timeout=600)
            dtr = time.perf_counter() - t0
            if r.returncode == 0:
                gbmp = os.path.join(tmp, "gpu.bmp")
                rt.write_bmp(gbmp, gpu_colors)
                res["ref_value"] = round(W * H * spp / dtr / 1e6, 3)
                res["ref_sample"] = (f"the reference's own main (main.c:107-305, sources under /root/reference built by "
                                     f"`make ref`, deterministic variant oracle/ref_unity.c), whole frame, "
                                     f"{REF_THREADS} threads, {dtr:.2f} s wall incl. OBJ load and BMP write")
                res["ref_bmp_equals_gpu_bmp"] = (hashlib.md5(open(bmp, "rb").read()).hexdigest() ==
                                                 hashlib.md5(open(gbmp, "rb").read()).hexdigest())
            else:
                res["ref_error"] = r.stderr[-300:]
    return res


# ---- roofline inputs committed under profiles/ ------------------------------------------------------------
def pmc_digest(workload, world):
    """profiles/pmc_<workload>.json (tools/pmc_digest.py over this workload's rocprofv3 runs): per kernel the
    rocprof average duration and per-dispatch counters -- VALU/SALU/LDS instructions, FP64 mix, LDS bank conflicts,
    FETCH_SIZE / WRITE_SIZE -- and which kernel the kernel trace names dominant."""
    path = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    try:
        dg = json.load(open(path))
    except Exception:
        return None
    return dg if dg.get("n_gpus", 1) == world else None


def kernel_roofline(name, live_ms, dg, work):
    """One kernel's roofline entry.  bound "valu": the path has no dense contraction (no MFMA) and its compulsory
    HBM traffic is tiny, so each kernel is held to its own VALU issue: wave-level VALU instructions x 2 cycles
    (FP64 x 4) over what 1024 SIMDs issue at 2.4 GHz in the measured time (valu_issue_frac); achieved / peak is the
    survey's algorithmic work (SURVEY.md §8 d: 57 flop per ray-triangle test) where the kernel does that work."""
    e = {"ms": round(live_ms, 4) if live_ms else None}
    k = (dg or {}).get("kernels", {}).get(name)
    if k:
        pd = k["per_dispatch"]
        valu = pd.get("SQ_INSTS_VALU")
        f64 = sum(pd.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        ms = live_ms or k.get("rocprof_avg_ms")
        if valu and ms:
            e["valu_insts_per_launch"] = int(valu)
            e["fp64_insts_per_launch"] = int(f64)
            e["valu_issue_frac"] = round((2.0 * valu + 2.0 * f64) / (1024 * ms * 1e-3 * 2.4e9), 4)
        gui = pd.get("GRBM_GUI_ACTIVE")
        if valu and gui:
            # the same issue slots over the kernel's own busy cycles in the PMC pass (rocprofv3 serialises dispatches
            # while it collects counters, so the kernel runs alone): GRBM_GUI_ACTIVE / 8 XCDs cycles per SIMD
            e["isolated_cycles"] = int(gui / 8)
            e["isolated_ms_at_2p4ghz"] = round(gui / 8 / 2.4e9 * 1e3, 4)
            e["valu_issue_frac_isolated"] = round((2.0 * valu + 2.0 * f64) / (1024 * gui / 8), 4)
        for c, key in (("SQ_INSTS_SALU", "salu_insts_per_launch"), ("SQ_INSTS_LDS", "lds_insts_per_launch"),
                       ("SQ_LDS_BANK_CONFLICT", "lds_bank_conflict_cycles_per_launch")):
            if c in pd:
                e[key] = int(pd[c])
        if "traffic_bytes" in k:
            e["traffic"] = k["traffic_bytes"]
            e["traffic_note"] = k.get("traffic_note")
            if ms:
                e["hbm_gbs"] = round(k["traffic_bytes"] / (ms * 1e-3) / 1e9, 2)
        e["rocprof_avg_ms"] = k.get("rocprof_avg_ms")
        e["source"] = dg.get("source")
    if work:
        e.update(work)
    return e


def frame_roofline(dg, frame_s):
    """The whole frame against both bounds: the VALU issue slots of every kernel of one frame (the
    digest's per-dispatch counters, one dispatch each) over what 1024 SIMDs issue at 2.4 GHz in ms_per_step, and the
    counter HBM bytes of those dispatches per frame against HBM_PEAK_GBS."""
    ks = (dg or {}).get("kernels") or {}
    if not ks or not frame_s:
        return None
    slots = bytes_ = 0.0
    names = []
    for name, k in sorted(ks.items()):
        pd = k.get("per_dispatch", {})
        if "SQ_INSTS_VALU" not in pd and "traffic_bytes" not in k:
            continue
        names.append(name)
        f64 = sum(pd.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        slots += 2.0 * pd.get("SQ_INSTS_VALU", 0) + 2.0 * f64
        bytes_ += k.get("traffic_bytes", 0)
    gbs = bytes_ / frame_s / 1e9
    return {"kernels": names, "valu_issue_frac": round(slots / (1024 * 2.4e9 * frame_s), 4),
            "bytes_per_frame": int(bytes_), "hbm_gbs": round(gbs, 2), "hbm_peak_gbs": HBM_PEAK_GBS,
            "hbm_frac": round(gbs / HBM_PEAK_GBS, 5), "source": dg.get("source")}


# ---- GPU ---------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="ultracomplex_1080p64", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-samples", type=float, default=1.4e8,
                    help="CPU baseline sample size (W*H*spp); the metric's config is rendered whole")
    ap.add_argument("--no-extras", action="store_true", help="skip the hoisted / no-tile-cull / latency extras")
    ap.add_argument("--band", default="auto",
                    help="N > 1 partition: rows per interleaved band (1: rows y = r + kN as main.c:84; 8: north_star's "
                         "row-tile split, bands of 8 rows).  auto: the faster one per frame size as measured on MI355X "
                         "(profiles/r05_*_rank_share_overlap.log, r05_f_scale*: 1080p rows (the 8-row bands' 1/8 shares "
                         "are less balanced: final tree 5.03x vs 4.47x), 4K bands of 8 (6.71x vs 6.68x, the mean of five "
                         "runs))")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: process group backend.  nccl (= RCCL, the default) needs a GPU per rank; gloo is an "
                         "explicit rehearsal mode in which ranks may share GPUs (no RCCL leg; the line then reports "
                         "the distinct GPUs used and ranks_per_gpu)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingc_amd as rt
    from raytracingc_amd.distributed import (SharedHostFrames, pin_rank_near_gpu, rank_config, rank_report,
                                             rows_per_rank)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    multi = world > 1
    if multi and args.backend == "nccl" and ndev < world:
        raise SystemExit(f"{world} ranks but {ndev} GPU(s): the nccl (RCCL) backend needs one GPU per rank; pass "
                         f"--backend gloo for a rehearsal with ranks sharing GPUs")
    gpu = local % ndev
    torch.cuda.set_device(gpu)
    # N > 1: the ranks share the node's CPU quota -- one intra-op thread each, pinned near their GPU when allowed
    pinning = pin_rank_near_gpu(gpu) if multi else None
    dev = torch.device("cuda", gpu)
    n_phys = min(world, ndev)  # distinct GPUs the ranks run on (one node)
    backend = None
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        backend = args.backend
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if multi:
            dist.barrier()

    def allreduce_max(v):
        if not multi:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def allreduce_sum(vals):
        if not multi:
            return vals
        t = torch.tensor(vals, dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t)
        return [int(v) for v in t.tolist()]

    scene_name, W, H, spp = WORKLOADS[args.workload]
    tris, tonly = load_scene(scene_name)
    scene = rt.default_scene()
    cam = rt.camera_basis()
    ds = rt.DeviceScene(tris, None, device=gpu)
    seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device=dev)
    band = (8 if H >= 2160 else 1) if args.band == "auto" else max(1, int(args.band))
    if world == 1:
        band = 1  # (a whole frame: no partition)
    rows = rows_per_rank(H, world, band)
    stream = torch.cuda.Stream(dev)
    nbuf = 3
    # this rank's compact rows of each frame in HBM; the host frames: pinned (N = 1) or node-shared (N > 1)
    dev_rows = [torch.zeros((rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    torch.cuda.synchronize(dev)  # (the zero fills ran on the current stream; the frames render on `stream`)
    shared = None
    if multi:
        shared = SharedHostFrames(f"rtc_bench_{os.environ.get('MASTER_PORT', '0')}", nbuf, H, W, local, barrier)
        host_ptr = [shared.rank_rows_ptr(b, rank, band) for b in range(nbuf)]
        host_frame = lambda b: shared.frames[b]  # noqa: E731
    else:
        host = [torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)]
        host_ptr = [h.data_ptr() + rank * W * 3 for h in host]
        host_frame = lambda b: host[b].numpy()  # noqa: E731
    pitch = world * band * W * 3  # between a rank's consecutive rows (bands) in the host frame

    cfg_joined = rt.RenderConfig(W, H, spp, 10, bool(tonly))
    cfg_r = rank_config(cfg_joined, rank, world, band)

    def loop(cfg, frames, cams=None):
        return ds.frame_loop(scene, cams or cam, cfg, [t.data_ptr() for t in dev_rows], host_ptr, pitch, frames,
                             stream.cuda_stream)

    local_s = [0.0]  # this rank's own time of the last timed region (rank_report)

    def timed(cfg, steps, warmup, cams=None):
        """warmup + steps pipelined frames (rtc_frame_loop: render with RTC_F_OVERLAP, each frame's rows copied into
        the host frame by the SDMA engines while the next frames render); the timed region spans the steps frames,
        barrier + device synchronisation on both sides, max over ranks."""
        if warmup:
            loop(cfg, warmup, cams)
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        st = loop(cfg, steps, cams)
        torch.cuda.synchronize(dev)
        barrier()
        local_s[0] = time.perf_counter() - t0
        dt = allreduce_max(local_s[0])
        return dt, st

    local_seg = [0] * rt.RTC_SEGMENT_COUNTERS  # this rank's own counters of the last counters() frame

    def counters(cfg):
        """the work counters of one more frame of the same configuration (untimed; every frame is identical)"""
        seg.zero_()
        ds.render_rows_async(scene, cam, cfg, dev_rows[0].data_ptr(), None, seg.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        local_seg[:] = [int(v) for v in seg.tolist()]
        return allreduce_sum(list(local_seg))

    # untimed frames for ~0.3 s: the GPU clocks settle before the kernel timing and the timed region
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < 0.3:
        loop(cfg_r, 10)
    # per-kernel device times of the split launch (HIP events the library records around rtc_render_chain on its
    # stream and around rtc_render_sky on the scene's side stream), averaged over frames launched like the timed ones
    # (RTC_F_OVERLAP: in-kernel sums, the cull streams), one at a time at settled clocks, like rocprofv3's kernel trace
    # of the same command
    kt = []
    cfg_t = dataclasses_replace(cfg_r, overlap=True)
    ds.set_timing(True)
    for _ in range(20):
        ds.render_rows_async(scene, cam, cfg_t, dev_rows[0].data_ptr(), None, None, stream.cuda_stream)
        k = ds.kernel_times()
        if k:
            kt.append(k)
    ds.set_timing(False)
    chain_ms = sky_ms = None
    if kt:
        chain_ms = allreduce_max(sum(a for a, _ in kt) / len(kt))
        sky_ms = allreduce_max(sum(b for _, b in kt) / len(kt))
    barrier()

    t, lst = timed(cfg_r, args.steps, args.warmup)
    seg_calls, seg_traced, tri_tests, cluster_tests, discarded_tests = counters(cfg_r)
    # N > 1: what the communicator reports (RCCL's rank count on the nccl backend) beside every rank's own ms and
    # segment count
    report = rank_report(local_s[0] / args.steps * 1e3, local_seg[0]) if multi else None
    samples = W * H * spp
    value = samples * args.steps / t / 1e6
    # the last frame of the timed run as it landed in host memory (every rank's rows)
    frame_host = host_frame((args.steps - 1) % nbuf).copy() if rank == 0 else None
    barrier()

    # a moving camera: the same pipelined frames (D2H included) over ORBIT_FRAMES distinct camera origins on an orbit
    # around the default look-at point, so every frame re-derives its primary records and the frame-to-frame reuse of
    # the static timed loop (the prep skip, the same-camera sky-pass wait elision) is never available
    orbit = orbit_cameras(rt)
    tm, _ = timed(cfg_r, args.steps, args.warmup, orbit)
    frame_mov = host_frame((args.steps - 1) % nbuf).copy() if rank == 0 else None
    barrier()
    moving = {"ms_per_step": round(tm / args.steps * 1e3, 4), "value": round(samples * args.steps / tm / 1e6, 3),
              "cameras": len(orbit),
              "what": f"{args.steps} pipelined frames, frame k from camera k mod {len(orbit)} of an orbit of "
                      f"+-{ORBIT_DEG:g} deg about the default look-at point (origins on a circle of the default "
                      "camera's distance), render + SDMA D2H into the host frame, like the headline loop"}

    extras = {}
    if multi and backend == "nccl":
        extras["rccl_device_frame"] = rccl_device_frame(args, tris, ds, scene, cam, cfg_r, rows, W, H, world, rank, dev, band,
                                                        barrier, allreduce_max)
    if not args.no_extras:
        # device-only frames (left in HBM), the bit-exact hoisted mode, the brute-force primary segments
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        cfg_o = dataclasses_replace(cfg_r, overlap=True)
        for k in range(args.steps):
            ds.render_rows_async(scene, cam, cfg_o, dev_rows[k % nbuf].data_ptr(), None, None, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        barrier()
        td = allreduce_max(time.perf_counter() - t0)
        extras["device_only"] = {"ms_per_step": round(td / args.steps * 1e3, 4),
                                 "value": round(samples * args.steps / td / 1e6, 3)}
        th, _ = timed(dataclasses_replace(cfg_r, hoist=True), args.steps, 1)
        _, ht, htests, _, _ = counters(dataclasses_replace(cfg_r, hoist=True))
        extras["hoisted"] = {"value": round(samples * args.steps / th / 1e6, 3),
                             "ms_per_step": round(th / args.steps * 1e3, 4), "segments_traced": ht,
                             "tri_tests": htests,
                             "bit_exact_vs_faithful": bool(rank != 0 or np.array_equal(
                                 host_frame((args.steps - 1) % nbuf), frame_host))}
        nb = max(2, args.steps // 4)
        tb, _ = timed(dataclasses_replace(cfg_r, tile_cull=False), nb, 1)
        _, _, btests, _, _ = counters(dataclasses_replace(cfg_r, tile_cull=False))
        extras["no_tile_cull"] = {"value": round(samples * nb / tb / 1e6, 3), "ms_per_step": round(tb / nb * 1e3, 4),
                                  "tri_tests": btests}
        # single-frame latency: render .. Color[] on the host, nothing overlapped (N = 1)
        if world == 1:
            lat = []
            for _ in range(5):
                torch.cuda.synchronize(dev)
                l0 = time.perf_counter()
                ds.render_rows_async(scene, cam, cfg_joined, dev_rows[0].data_ptr(), None, None, stream.cuda_stream)
                stream.synchronize()
                rt.copy_d2h_dma(host_ptr[0], dev_rows[0].data_ptr(), H * W * 3)
                lat.append((time.perf_counter() - l0) * 1e3)
            extras["frame_latency_ms"] = round(sorted(lat)[len(lat) // 2], 4)

    if rank == 0:
        T = len(tris)
        tests_per_launch = tri_tests / world
        dg = pmc_digest(args.workload, world)
        chain_work = None
        if chain_ms:
            ach = tests_per_launch * FLOPS_PER_TEST / (chain_ms * 1e-3) / 1e12
            chain_work = {"achieved_tflops": round(ach, 3), "peak_tflops": FP32_VALU_PEAK_TFLOPS,
                          "frac_57flop": round(ach / FP32_VALU_PEAK_TFLOPS, 4),
                          "work_per_launch": f"{tests_per_launch:.4g} ray-triangle tests x {FLOPS_PER_TEST} flop"}
        kernels = {"rtc_render_chain": kernel_roofline("rtc_render_chain", chain_ms, dg, chain_work),
                   "rtc_render_sky": kernel_roofline("rtc_render_sky", sky_ms, dg, {
                       "work_per_launch": "getEnvironmentLight (raytracing.c:151-160) once per sample of every pixel "
                                          "whose primary ray misses: 2 glibc powf + 2 smoothstep (f64 tails)"})}
        dominant = (dg or {}).get("dominant") or max(kernels, key=lambda k: kernels[k].get("ms") or 0)
        dk = kernels[dominant]
        # the line's top-level roofline: the dominant kernel against its VALU issue bound (no MFMA, no HBM bound)
        frac = dk.get("valu_issue_frac")
        bf_tf = seg_traced / world * T * FLOPS_PER_TEST / (t / args.steps) / 1e12
        frame_roof = frame_roofline(dg, t / args.steps)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": n_phys,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"reference scene {scene_name}.obj (Triangle[] from the reference loader, tests/golden/scenes), "
                    "default camera/sky/sun, per-pixel seed x+y*W",
            "config": {"workload": args.workload, "scene": f"{scene_name}.obj", "width": W, "height": H, "spp": spp,
                       "max_bounce": 10, "triangles": T, "row_band": band, "chain_wgs_per_cu": ds.chain_wgs,
                       "parallelism": (f"rows mod {world}" if band == 1 else
                                       f"bands of {band} rows mod {world} (row-tile split)")
                                      + "; each rank SDMA-copies its rows into the shared host frame"
                                      + ("; RCCL gather to rank 0's GPU measured beside it (rccl_device_frame)"
                                         if backend == "nccl" else "")
                                      + (f"; REHEARSAL: {world} gloo ranks on {n_phys} GPU(s), no RCCL leg, not a "
                                         "scaling measurement" if backend == "gloo" else ""),
                       "step": "render + D2H of Color[W*H] into pinned host memory (rtc_frame_loop: frames pipelined, "
                               "frame k+1's preparation overlapping frame k's sky pass; frame k's SDMA copy overlapping "
                               "the next frames' renders; triple-buffered)",
                       "mode": "faithful (every sample re-traces its primary ray and every miss evaluates the "
                               "environment)"},
            "roofline": {"bound": "valu", "dominant": dominant,
                         "achieved": dk.get("valu_issue_frac"), "peak": 1.0, "unit": "VALU issue fraction",
                         "frac": frac, "frac_isolated": dk.get("valu_issue_frac_isolated"),
                         "traffic": dk.get("traffic"),
                         # SURVEY §8(d)'s own contract: executed ray-triangle tests x 57 flop over the chain kernel's
                         # time against the FP32 vector peak
                         "frac_57flop": (chain_work or {}).get("frac_57flop"),
                         "frame": frame_roof,
                         "kernels": kernels,
                         "bruteforce_equiv_tflops": round(bf_tf, 3),
                         "note": "per kernel: ms = HIP events around it on its own stream (live); valu_issue_frac = "
                                 "(2 x VALU + 2 x FP64 wave instructions) / (1024 SIMDs x 2.4 GHz x ms), the span-based "
                                 "fraction; valu_issue_frac_isolated = the same over GRBM_GUI_ACTIVE / 8 XCDs cycles of "
                                 "the kernel's own dispatch in the PMC pass (it runs alone there); counters from "
                                 "the committed rocprofv3 PMC digest of this workload (roofline.kernels.*.source); "
                                 "frac_57flop = ray-triangle tests x 57 flop / ms / 157.3 TFLOP/s (SURVEY §8 d); "
                                 "traffic = counter HBM bytes per launch (traffic_note: which correction); "
                                 "bruteforce_equiv = segments x T x 57 per frame time, not a roofline; frame = every "
                                 "kernel of one frame (the digest's per-dispatch counters) over ms_per_step: VALU issue "
                                 "and counter HBM bytes against 8 TB/s (north_star's HBM roofline fraction)"},
            "frame_ms": round(t / args.steps * 1e3, 4),
            "frame_loop": {"enqueue_ms_per_frame": round(lst["enqueue_ms"] / max(1, lst["frames"]), 4),
                           "copy_ms_median": round(lst["copy_ms_median"], 4), "copy_ms_max": round(lst["copy_ms_max"], 4),
                           "d2h": "rtc_copy_rows_d2h_dma (SDMA engines, the CPU agent nearest the GPU), native copy "
                                  "thread"},
            "segments_per_frame": seg_calls,
            "segments_traced_per_frame": seg_traced,
            "msegments_per_s": round(seg_traced * args.steps / t / 1e6, 2),
            "tri_tests_per_frame": tri_tests,
            "discarded_tri_tests_per_frame": discarded_tests,
            "gtests_per_s": round(tri_tests * args.steps / t / 1e9, 2),
        }
        # the frame as it landed in host memory == one GPU rendering the whole frame through rtc_render
        ref1, gacc, _ = rt.render(tris, None, scene, cam, cfg_joined, device=gpu, want_accum=(world == 1))
        line["host_frame_equals_rtc_render"] = bool(np.array_equal(frame_host, ref1))
        if multi:
            line["rank_cpu"] = pinning
            line["ranks"] = world
            line["ranks_per_gpu"] = round(world / n_phys, 3)
            line["rehearsal"] = backend == "gloo"
            line["ranks_report"] = report
            if backend == "nccl":
                line["rccl_nranks"] = report["comm_world_size"]
        mcam = orbit[(args.steps - 1) % len(orbit)]
        refm, _, _ = rt.render(tris, None, scene, mcam, cfg_joined, device=gpu)
        moving["last_frame_equals_rtc_render"] = bool(np.array_equal(frame_mov, refm))
        line["moving_camera"] = moving
        line.update(extras)
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(tris, tonly, scene, cam, W, H, spp, args.cpu_budget_samples, frame_host, gacc)
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(line), flush=True)
    barrier()
    ds.close()
    if shared is not None:
        shared.close(barrier)
    if multi:
        dist.destroy_process_group()


ORBIT_FRAMES, ORBIT_DEG = 20, 15.0


def orbit_cameras(rt):
    """ORBIT_FRAMES cameras (main.c:252-255 bases) whose origins sweep +-ORBIT_DEG degrees about the default look-at
    point in the horizontal plane, at the default camera's distance and height."""
    ox, oy, oz = rt.DEFAULT_ORIGIN
    lx, ly, lz = rt.DEFAULT_LOOKING_AT
    r = math.hypot(ox - lx, oz - lz)
    a0 = math.atan2(oz - lz, ox - lx)
    cams = []
    for k in range(ORBIT_FRAMES):
        a = a0 + math.radians(-ORBIT_DEG + 2 * ORBIT_DEG * k / (ORBIT_FRAMES - 1))
        cams.append(rt.camera_basis((lx + r * math.cos(a), oy, lz + r * math.sin(a)), rt.DEFAULT_LOOKING_AT,
                                    rt.DEFAULT_FOV))
    return cams


def dataclasses_replace(cfg, **kw):
    import dataclasses

    return dataclasses.replace(cfg, **kw)


def rccl_device_frame(args, tris, ds, scene, cam, cfg_r, rows, W, H, world, rank, dev, band, barrier, allreduce_max):
    """N > 1, every rank on its own GPU: the device-frame path -- each frame's parts gathered to rank 0's GPU over
    xGMI (torch.distributed `nccl` = RCCL) and re-interleaved there (rtc_deinterleave_async), pipelined like the
    host-frame loop (render on one stream, the gather on another after the frame event).  Returns its timing and
    whether the gathered frame equals the single-GPU render."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingc_amd as rt

    nbuf = 3
    stream, gst = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    parts = [torch.zeros((rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    gathered = [torch.zeros((world, rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if rank == 0 else None
    frames = [torch.zeros((H, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if rank == 0 else None
    free = [None] * nbuf
    cfg_o = dataclasses_replace(cfg_r, overlap=True)

    def step(k):
        b = k % nbuf
        if free[b] is not None:
            stream.wait_event(free[b])
        ready = torch.cuda.Event()
        ready.record(stream)
        ds.set_frame_event(ready.cuda_event)
        ds.render_rows_async(scene, cam, cfg_o, parts[b].data_ptr(), None, None, stream.cuda_stream)
        gst.wait_event(ready)
        with torch.cuda.stream(gst):
            dist.gather(parts[b], gather_list=list(gathered[b].unbind(0)) if rank == 0 else None, dst=0)
            if rank == 0:
                rt.deinterleave_async(gathered[b].data_ptr(), world, rows, W, H, frames[b].data_ptr(), gst.cuda_stream,
                                      band)
        done = torch.cuda.Event()
        done.record(gst)
        free[b] = done

    for k in range(args.warmup):
        step(k)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    barrier()
    t = allreduce_max(time.perf_counter() - t0)
    out = {"ms_per_step": round(t / args.steps * 1e3, 4),
           "value": round(W * H * cfg_r.spp * args.steps / t / 1e6, 3),
           "what": "frame gathered into rank 0's HBM over RCCL (ncclGather via torch.distributed) and re-interleaved; "
                   "no D2H"}
    if rank == 0:
        ref1, _, _ = rt.render(tris, None, scene, cam, dataclasses_replace(cfg_r, row_start=0, row_stride=1, row_band=0),
                               device=dev.index)
        out["frame_equals_1gpu_render"] = bool(np.array_equal(frames[(args.steps - 1) % nbuf].cpu().numpy(), ref1))
    return out


if __name__ == "__main__":
    main()

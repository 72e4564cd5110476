#!/usr/bin/env python3
"""Benchmark: Mrays/s + frame time of the MI355X render path on BASELINE.json's workload.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ultracomplex_1080p64|...]

A step = one frame, timed as SURVEY.md §8(d) / BASELINE.md §3 define it: from the render launch until the
frame's Color[W*H] is in host memory (the buffer main.c:305 hands to stbi_write_bmp).  Every rank renders its
interleaved rows (y = rank + k*N, main.c:84 lifted to GPUs) with the HIP kernels, the uint8 parts are gathered
to rank 0 over RCCL (torch.distributed `nccl`) and re-interleaved there, and rank 0 copies the frame into pinned
host memory (hipMemcpyAsync on a copy stream; frame k's copy overlaps frame k+1's render, double-buffered).
The scene (the reference loader's Triangle[], tests/golden/scenes) is resident in HBM before timing.

Prints ONE JSON line on rank 0.  `value` = W*H*spp*K / t / 1e6 over the whole job (strong scaling: the frame is
fixed, N GPUs split it).  `roofline` is the dominant (heavy-tile) kernel against the FP32 VALU peak with the
survey's algorithmic 57 flop per ray-triangle test (SURVEY.md §8 d); `cpu_baseline` is the CPU restatement of
the reference (oracle/, "port") on the same workload on the box's host cores, beside the reference itself
compiled here (oracle/_ref/rtc_ref), rank 0 at N = 1 only.
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
    reference on every golden fixture; gcc -O3, no FMA) with row-interleaved pthreads like main.c:84 at
    threads = nproc and at the reference's 12, plus the reference's own sources compiled here
    (oracle/_ref/rtc_ref, 12 threads, its own main) when the whole frame fits the budget.  Rows
    y = 0, s, 2s, ... of the same frame with s = ceil(samples / budget) (s = 1 at the metric's config)."""
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
    dt, ccol, cacc, seg = run(n_all)
    dt12, _, _, _ = run(REF_THREADS)
    rows = ccol.shape[0]
    samples = rows * W * spp
    res = {
        "value": samples / dt / 1e6, "unit": "Mrays/s", "cores": n_all, "kind": "port",
        "threads": n_all, "value_12t": round(samples / dt12 / 1e6, 3),
        "cpu_model": info.get("model"),
        "topology": f"{info.get('sockets')} sockets x {info.get('cores_per_socket')} cores x "
                    f"{info.get('threads_per_core')} SMT = nproc {info['nproc']}; affinity {info['affinity']} CPUs, "
                    f"cgroup quota {info.get('cgroup_cpus')} CPUs",
        "sample": (f"{'the whole frame' if stride == 1 else f'rows y = 0 mod {stride} of the frame'} ({rows} rows x "
                   f"{W} x {spp} spp = {samples} samples, {seg} segments), render loop only: {dt:.2f} s on {n_all} "
                   f"threads, {dt12:.2f} s on {REF_THREADS}; oracle/rtc_oracle.c (gcc -O3, no FMA)"),
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
    ap.add_argument("--d2h", default="dma", choices=["dma", "kernel", "runtime"],
                    help="how Color[] reaches host memory: the SDMA engines (rtc_copy_d2h_dma), a 32-workgroup copy "
                         "kernel (rtc_copy_async) or hipMemcpyAsync")
    ap.add_argument("--no-overlap", action="store_true",
                    help="join every frame's sky pass into the render stream (no frame pipelining)")
    ap.add_argument("--no-extras", action="store_true", help="skip the hoisted / no-tile-cull / latency extras")
    ap.add_argument("--force-gather", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--diag-repeat", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingc_amd as rt
    from raytracingc_amd.distributed import rank_config, rows_per_rank

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # --force-gather: the multi-GPU data path (per-rank parts, RCCL gather on its own stream, re-interleave) with a
    # single rank -- its streams, events and RCCL calls exercised on a one-GPU box (RCCL refuses two ranks on one
    # device, so N > 1 itself cannot be rehearsed there)
    multi = world > 1 or args.force_gather
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    scene_name, W, H, spp = WORKLOADS[args.workload]
    tris, tonly = load_scene(scene_name)
    scene = rt.default_scene()
    cam = rt.camera_basis()
    ds = rt.DeviceScene(tris, None, device=local)
    seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device=dev)
    rows = rows_per_rank(H, world)
    # the frames render on a non-blocking stream of their own (not the legacy default stream, whose implicit
    # synchronisation with other streams costs the overlapped D2H); the copies on a second one
    stream = torch.cuda.Stream(dev)
    copy_stream = torch.cuda.Stream(dev)
    gather_stream = torch.cuda.Stream(dev)  # N > 1: RCCL gather + re-interleave of each frame, after its render
    # three frame buffers: frame k+2 renders while frame k's D2H (issued at frame k+1's geometry-done event) may
    # still be in flight, so the copy is off the render's critical path
    nbuf = 3
    parts = [torch.zeros((rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if multi else None
    gathered = ([torch.zeros((world, rows, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
                if (multi and rank == 0) else None)
    part_free = [None] * nbuf  # N > 1: parts[b]'s previous gather has finished
    frames = [torch.zeros((H, W, 3), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if rank == 0 else None
    host = [torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)] if rank == 0 else None

    # the library records geo_ev on the render stream once a frame's geometry-pixel kernels are enqueued
    # (rtc_scene_set_geometry_event): the previous frame's D2H starts there, overlapping this frame's sky pass
    # rather than the start of its persistent geometry kernel (a blit kernel holding CU slots then would delay
    # some of that kernel's workgroups for the whole copy)
    geo_ev = torch.cuda.Event()
    geo_ev.record(stream)
    torch.cuda.synchronize(dev)
    ds.set_geometry_event(geo_ev.cuda_event)

    def render_step(cfg, b, count=False):
        """One frame into device frame buffer b (rank 0: rendered, or gathered and re-interleaved); returns the
        event at which frame buffer b holds the whole frame.  The library records the frame event once both of
        its passes are written (rtc_scene_set_frame_event: after the join, or with cfg.overlap -- frame
        pipelining, the next frame's preparation overlapping this one's sky pass -- on its side stream); the
        gather (RCCL, N > 1) and the D2H wait for it.  count: the kernels also add into the segment counters
        (instrumentation: a separate untimed frame)."""
        cfg_r = rank_config(cfg, rank, world)
        segp = seg.data_ptr() if count else None
        ready = torch.cuda.Event()
        ready.record(stream)  # creates the hipEvent_t (a torch event has none before its first record)
        # the library records the frame event while enqueuing the launch; it is cleared right after, so that no
        # later launch records an event this function's caller may already have released
        ds.set_frame_event(ready.cuda_event)
        if not multi:
            ds.render_rows_async(scene, cam, cfg_r, frames[b].data_ptr(), None, segp, stream.cuda_stream)
            ds.set_frame_event(None)
            return ready
        if part_free[b] is not None:  # parts[b] is rewritten once its previous gather has read it
            stream.wait_event(part_free[b])
        ds.render_rows_async(scene, cam, cfg_r, parts[b].data_ptr(), None, segp, stream.cuda_stream)
        ds.set_frame_event(None)
        gather_stream.wait_event(ready)
        with torch.cuda.stream(gather_stream):  # the gather (RCCL) orders itself after the frame on this stream
            dist.gather(parts[b], gather_list=list(gathered[b].unbind(0)) if rank == 0 else None, dst=0)
            if rank == 0:
                rt.deinterleave_async(gathered[b].data_ptr(), world, rows, W, H, frames[b].data_ptr(),
                                      gather_stream.cuda_stream)
        done = torch.cuda.Event()
        done.record(gather_stream)
        part_free[b] = done
        return done

    nbytes = H * W * 3

    def d2h_now(b, st):
        """The D2H of frame buffer b into pinned host buffer b, ordered after the work enqueued on stream st so
        far; returns when it is done (dma) or enqueued on st (kernel, runtime)."""
        if args.d2h == "dma":
            st.synchronize()
            rt.copy_d2h_dma(host[b].data_ptr(), frames[b].data_ptr(), nbytes)
        elif args.d2h == "kernel":
            rt.copy_async(host[b].data_ptr(), frames[b].data_ptr(), nbytes, 32, st.cuda_stream)
        else:
            with torch.cuda.stream(st):
                host[b].copy_(frames[b], non_blocking=True)

    copy_ms = []  # dma: each frame copy's duration as the copying thread saw it (the last run)

    def run(cfg, steps, warmup, d2h=True):
        """warmup + steps frames; the timed region spans the steps frames, each rendered and (rank 0, d2h) copied
        into pinned host memory, the copy of frame k overlapping the renders of the next frames:
          dma     the SDMA engines (rtc_copy_d2h_dma) from a host thread that waits for frame k's event;
          kernel  a 32-workgroup copy kernel (rtc_copy_async) on a copy stream, from frame k+1's geometry-done
                  event (rtc_scene_set_geometry_event) so that it overlaps frame k+1's sky pass;
          runtime hipMemcpyAsync (the runtime's blit kernel), likewise.
        Frame buffer b is reused only once its previous copy has finished."""
        use_d2h = d2h and rank == 0
        copy_ms.clear()
        if use_d2h and args.d2h == "dma":
            jobs = queue.Queue()
            free = [threading.Event() for _ in range(nbuf)]
            for e in free:
                e.set()
            err = []

            def worker():
                while True:
                    job = jobs.get()
                    if job is None:
                        return
                    b, ev = job
                    try:
                        ev.synchronize()
                        c0 = time.perf_counter()
                        rt.copy_d2h_dma(host[b].data_ptr(), frames[b].data_ptr(), nbytes)
                        copy_ms.append((time.perf_counter() - c0) * 1e3)
                    except Exception as e:  # surfaced by the main thread
                        err.append(e)
                    free[b].set()

            def frames_loop(n):
                th = threading.Thread(target=worker, daemon=True)
                th.start()
                for k in range(n):
                    b = k % nbuf
                    free[b].wait()
                    free[b].clear()
                    jobs.put((b, render_step(cfg, b)))
                jobs.put(None)
                th.join()
                if err:
                    raise err[0]
        else:
            copied = [None] * nbuf

            def copy_after(b, *after):
                for e in after:
                    copy_stream.wait_event(e)
                d2h_now(b, copy_stream)
                done = torch.cuda.Event()
                done.record(copy_stream)
                return done

            def frames_loop(n):
                pending = None
                for k in range(n):
                    b = k % nbuf
                    if copied[b] is not None:  # frame buffer b is free once its previous D2H has finished
                        stream.wait_event(copied[b])
                        gather_stream.wait_event(copied[b])
                    ready = render_step(cfg, b)
                    if use_d2h:
                        if pending is not None:
                            copied[pending[0]] = copy_after(pending[0], pending[1], geo_ev)
                        pending = (b, ready)
                if use_d2h and pending is not None:
                    copied[pending[0]] = copy_after(pending[0], pending[1])

        frames_loop(warmup)
        if multi:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        frames_loop(steps)
        torch.cuda.synchronize(dev)
        if multi:
            dist.barrier()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        if multi:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # the work counters of one more frame of the same configuration (untimed; every frame is identical)
        seg.zero_()
        render_step(cfg, 0, count=True)
        torch.cuda.synchronize(dev)
        segs = seg.clone()
        if multi:
            dist.all_reduce(segs)
        return float(t[0]), [int(v) for v in segs.tolist()]

    # the timed frames are pipelined (RenderConfig.overlap, RTC_F_OVERLAP: frame k+1's preparation overlaps frame
    # k's sky pass; same frames) unless --no-overlap; the settle, kernel-timing and latency frames are joined
    cfg_joined = rt.RenderConfig(W, H, spp, 10, bool(tonly))
    cfg = rt.RenderConfig(W, H, spp, 10, bool(tonly), overlap=not args.no_overlap)
    # untimed frames for ~0.3 s: the GPU clocks settle before the kernel timing, the warmup and the timed region
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < 0.3:
        for k in range(10):
            ds.render_rows_async(scene, cam, rank_config(cfg_joined, rank, world),
                                 (parts[0] if multi else frames[0]).data_ptr(), None, None, stream.cuda_stream)
            if rank == 0:  # the pinned buffers' first copies are slow (mapping): make them here, untimed
                d2h_now(k % nbuf, stream)
        torch.cuda.synchronize(dev)
    # per-kernel device times of the split launch (HIP events the library records around the geometry-pixel
    # kernel on this stream and around the sky kernel on the scene's side stream), averaged over frames rendered
    # back to back at settled clocks, like rocprofv3's kernel trace of the same command
    heavy_ms = sky_ms = None
    kt = []
    ds.set_timing(True)
    for _ in range(20):
        ds.render_rows_async(scene, cam, rank_config(cfg_joined, rank, world), (parts[0] if multi else frames[0]).data_ptr(),
                             None, None, stream.cuda_stream)
        k = ds.kernel_times()
        if k:
            kt.append(k)
    ds.set_timing(False)
    if kt:
        hk = torch.tensor([sum(a for a, _ in kt) / len(kt), sum(b for _, b in kt) / len(kt)], dtype=torch.float64,
                          device=dev)
        if multi:
            dist.all_reduce(hk, op=dist.ReduceOp.MAX)
        heavy_ms, sky_ms = float(hk[0]), float(hk[1])
    if multi:
        dist.barrier()

    if args.diag_repeat:  # diagnosis only: the same timed run a few times before the reported one
        print(json.dumps({"diag_repeat_ms": [round(run(cfg, args.steps, args.warmup)[0] / args.steps * 1e3, 4)
                                             for _ in range(args.diag_repeat)]}), flush=True)
    t, (seg_calls, seg_traced, tri_tests, cluster_tests, discarded_tests) = run(cfg, args.steps, args.warmup)
    samples = W * H * spp
    value = samples * args.steps / t / 1e6
    # the last frame of the timed run as it landed in host memory
    host_frame = host[(args.steps - 1) % nbuf].numpy().copy() if rank == 0 else None
    # the D2H of one frame: dma -- the median copy of the timed run (SDMA, overlapping the next frames' renders);
    # kernel / runtime -- ten copies on their own after it
    d2h_ms = None
    if rank == 0 and args.d2h == "dma" and copy_ms:
        d2h_ms = sorted(copy_ms)[len(copy_ms) // 2]
    elif rank == 0:
        torch.cuda.synchronize(dev)
        c0 = time.perf_counter()
        for k in range(10):
            d2h_now(k % nbuf, copy_stream)
        copy_stream.synchronize()
        d2h_ms = (time.perf_counter() - c0) / 10 * 1e3

    extras = {}
    if not args.no_extras:
        # device-only frames (no D2H), the bit-exact hoisted mode and the brute-force primary segments
        td, _ = run(cfg, args.steps, 1, d2h=False)
        extras["device_only"] = {"ms_per_step": round(td / args.steps * 1e3, 4),
                                 "value": round(samples * args.steps / td / 1e6, 3)}
        ref_frame = frames[0].clone() if rank == 0 else None
        th, (_, ht, htests, _, _) = run(rt.RenderConfig(W, H, spp, 10, bool(tonly), hoist=True, overlap=cfg.overlap), args.steps, 1)
        extras["hoisted"] = {"value": round(samples * args.steps / th / 1e6, 3),
                             "ms_per_step": round(th / args.steps * 1e3, 4), "segments_traced": ht,
                             "tri_tests": htests,
                             "bit_exact_vs_faithful": bool(rank != 0 or torch.equal(frames[0], ref_frame))}
        nb = max(2, args.steps // 4)
        tb, (_, _, btests, _, _) = run(rt.RenderConfig(W, H, spp, 10, bool(tonly), tile_cull=False), nb, 1)
        extras["no_tile_cull"] = {"value": round(samples * nb / tb / 1e6, 3), "ms_per_step": round(tb / nb * 1e3, 4),
                                  "tri_tests": btests}
        # single-frame latency: render .. Color[] on the host, nothing overlapped
        if rank == 0 and world == 1:
            lat = []
            for _ in range(5):
                torch.cuda.synchronize(dev)
                l0 = time.perf_counter()
                ds.render_rows_async(scene, cam, cfg_joined, frames[0].data_ptr(), None, None, stream.cuda_stream)
                d2h_now(0, stream)
                stream.synchronize()
                lat.append((time.perf_counter() - l0) * 1e3)
            extras["frame_latency_ms"] = round(sorted(lat)[len(lat) // 2], 4)

    if rank == 0:
        T = len(tris)
        tests_per_launch = tri_tests / world
        dom_ms = heavy_ms if heavy_ms else t / args.steps * 1e3
        achieved_tf = tests_per_launch * FLOPS_PER_TEST / (dom_ms * 1e-3) / 1e12
        bf_tf = seg_traced / world * T * FLOPS_PER_TEST / (t / args.steps) / 1e12
        traffic = None
        pmc_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            try:
                pm = json.load(open(pmc_path)).get(args.workload)
                if pm and pm.get("n_gpus", 1) == world:
                    traffic = pm["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
        # VALU issue of the dominant kernel (profiles/r02_e_pmc_breakdown.json: rocprofv3 SQ counters of one launch of
        # this workload): wave-level VALU instructions x 2 cycles (FP64 x 4) over what 1024 SIMDs (256 CUs x 4)
        # issue at 2.4 GHz in the measured kernel time -- how close the kernel runs to its own issue bound
        issue = None
        brk = os.path.join(REPO, "profiles", "r02_e_pmc_breakdown.json")
        if os.path.exists(brk) and args.workload == "ultracomplex_1080p64" and world == 1:
            try:
                pd = json.load(open(brk))["rtc_render_chain"]["_per_dispatch"]
                f64 = pd["SQ_INSTS_VALU_ADD_F64"] + pd["SQ_INSTS_VALU_MUL_F64"] + pd["SQ_INSTS_VALU_FMA_F64"] + \
                    pd["SQ_INSTS_VALU_TRANS_F64"]
                cyc = 2.0 * pd["SQ_INSTS_VALU"] + 2.0 * f64
                issue = {"valu_insts_per_launch": int(pd["SQ_INSTS_VALU"]), "fp64_insts_per_launch": int(f64),
                         "salu_insts_per_launch": int(pd["SQ_INSTS_SALU"]),
                         "valu_issue_frac": round(cyc / (1024 * dom_ms * 1e-3 * 2.4e9), 4),
                         "source": "profiles/r02_e_pmc_breakdown.json"}
            except Exception:
                issue = None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
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
                       "max_bounce": 10, "triangles": T, "parallelism": f"rows mod {world} + RCCL gather",
                       "step": "render + gather + re-interleave + D2H of Color[W*H] into pinned host memory "
                               "(triple-buffered: frame k's D2H overlaps the next frames' renders; d2h_method)"
                               + ("; frames pipelined: frame k+1's primary records and tile cull overlap frame k's "
                                  "sky pass (RTC_F_OVERLAP), its geometry kernel starts after it" if cfg.overlap else
                                  "; frames joined (--no-overlap)"),
                       "mode": "faithful (every sample re-traces its primary ray and every miss evaluates the "
                               "environment)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": FP32_VALU_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_VALU_PEAK_TFLOPS, 4),
                         "traffic": traffic,
                         "kernel": "rtc_render_chain (geometry pixels of the split launch; state-indexed samples)",
                         "kernel_ms": round(dom_ms, 4),
                         "sky_kernel_ms": round(sky_ms, 4) if sky_ms else None,
                         "work_per_launch": f"{tests_per_launch:.4g} ray-triangle tests x {FLOPS_PER_TEST} flop",
                         "cluster_tests_per_launch": cluster_tests // world,
                         "hbm_achieved_gbs": (round(traffic / (dom_ms * 1e-3) / 1e9, 3) if traffic else None),
                         "hbm_peak_gbs": HBM_PEAK_GBS,
                         "bruteforce_equiv_tflops": round(bf_tf, 3),
                         "issue": issue,
                         "note": "achieved: the ray-triangle tests the kernel evaluated x 57 flop / its device time "
                                 "(HIP events around it on the launch stream); traffic: rocprofv3 FETCH_SIZE x 2 + "
                                 "WRITE_SIZE per launch (profiles/pmc_traffic.json); hbm_achieved_gbs: traffic / "
                                 "kernel time; bruteforce_equiv: segments x T (the reference's brute-force work) per "
                                 "frame time"},
            "frame_ms": round(t / args.steps * 1e3, 4),
            "d2h_method": {"dma": "rtc_copy_d2h_dma (SDMA engines, host copy thread)",
                           "kernel": "rtc_copy_async (32 workgroups, copy stream)",
                           "runtime": "hipMemcpyAsync (runtime blit kernel, copy stream)"}[args.d2h],
            "host_frame_equals_device_frame": bool(rank != 0 or torch.equal(torch.from_numpy(host_frame),
                                                                             frames[(args.steps - 1) % nbuf].cpu())),
            "d2h_ms": round(d2h_ms, 4) if d2h_ms is not None else None,
            "segments_per_frame": seg_calls,
            "segments_traced_per_frame": seg_traced,
            "msegments_per_s": round(seg_traced * args.steps / t / 1e6, 2),
            "tri_tests_per_frame": tri_tests,
            "discarded_tri_tests_per_frame": discarded_tests,
            "gtests_per_s": round(tri_tests * args.steps / t / 1e9, 2),
        }
        if multi:
            # the gathered, re-interleaved frame as it landed on the host == one GPU rendering the whole frame
            ref1, _, _ = rt.render(tris, None, scene, cam, cfg_joined, device=local)
            line["frame_equals_1gpu_render"] = bool(np.array_equal(host_frame, ref1))
        line.update(extras)
        if world == 1 and not args.no_cpu_baseline:
            # the GPU's float frame for the bit comparison (one more render through the C ABI)
            _, gacc, _ = rt.render(tris, None, scene, cam, cfg_joined, device=local, want_accum=True)
            cb = cpu_baseline(tris, tonly, scene, cam, W, H, spp, args.cpu_budget_samples, host_frame, gacc)
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(line), flush=True)
    ds.close()
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: Mrays/s + frame time of the MI355X render path on BASELINE.json's workload.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ultracomplex_1080p64|ultracomplex_4k64]

A step = one frame: every rank renders its interleaved rows (y = rank + k*N, main.c:84 lifted to GPUs) with
the HIP kernel, the uint8 parts are gathered to rank 0 over RCCL (torch.distributed `nccl`) and re-interleaved
on rank 0.  The scene (ultracomplex.obj as the reference's loader produced it, tests/golden/scenes) is resident
in HBM before timing; outputs stay in HBM (the D2H of the finished frame is reported separately).

Prints ONE JSON line on rank 0.  `value` = W*H*spp*K / t / 1e6 over the whole job (strong scaling: the frame
is fixed, N GPUs split it).  `roofline` is the dominant (render) kernel against the FP32 VALU peak with the
survey's algorithmic 57 flop per ray-triangle test (SURVEY.md §8 d); `cpu_baseline` is the CPU restatement
of the reference (oracle/, "port") on a bounded row sample of the same frame, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mrays/sec + frame time, 1920x1080x64spp ultracomplex.obj, 1/2/4/8 GPUs"
FP32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (FP32 vector, spec)
HBM_PEAK_GBS = 8000.0
FLOPS_PER_TEST = 57  # full rayTriangle path
WORKLOADS = {
    "ultracomplex_1080p64": ("ultracomplex", 1920, 1080, 64),
    "ultracomplex_4k64": ("ultracomplex", 3840, 2160, 64),
    "fsuzane_1080p64": ("fsuzane", 1920, 1080, 64),
    "cube_1080p16": ("cube", 1920, 1080, 16),
}


def load_scene(name):
    import numpy as np

    from raytracingc_amd import TRIANGLE_DT

    raw = open(os.path.join(REPO, "tests", "golden", "scenes", name + ".tris"), "rb").read()
    count, tonly = np.frombuffer(raw[:8], np.int32)
    return np.frombuffer(raw[8:8 + 68 * int(count)], TRIANGLE_DT).copy(), int(tonly)


def cpu_baseline(tris, tonly, scene, cam, W, H, spp, row_stride):
    """The reference algorithm on the host (oracle/rtc_oracle.c, bit-identical to the reference on the golden
    fixtures) over rows y = 0, s, 2s, ... of the same frame.  Threads = the box's CPU share (<= 16)."""
    import oracle.binding as orc
    from raytracingc_amd._abi import RtcRenderDesc

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    d = RtcRenderDesc(W, H, spp, 10, tonly, 0, row_stride, 0)
    t0 = time.perf_counter()
    colors, _, seg = orc.render(tris, None, scene, cam, d, threads=threads)
    dt = time.perf_counter() - t0
    rows = colors.shape[0]
    samples = rows * W * spp
    return {
        "value": samples / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
        "sample": f"rows y=0 mod {row_stride} of the same frame ({rows} rows x {W} x {spp} spp = {samples} samples, "
                  f"{seg} segments), {dt:.2f} s wall on {threads} threads; oracle/rtc_oracle.c (gcc -O3, no FMA)",
        "seconds": dt,
    }, colors


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="ultracomplex_1080p64", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-row-stride", type=int, default=4)
    ap.add_argument("--no-hoisted", action="store_true", help="skip the extra hoisted-mode measurement")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingc_amd as rt
    from raytracingc_amd.distributed import FrameRenderer, hip_part_renderer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    scene_name, W, H, spp = WORKLOADS[args.workload]
    tris, tonly = load_scene(scene_name)
    scene = rt.default_scene()
    cam = rt.camera_basis()
    ds = rt.DeviceScene(tris, None, device=local)
    seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device=dev)

    def make(hoist, tile_cull=True):
        cfg = rt.RenderConfig(W, H, spp, 10, bool(tonly), hoist, tile_cull=tile_cull)
        return FrameRenderer(cfg, hip_part_renderer(ds, scene, cam, seg), dev)

    def run(fr, steps, warmup):
        stream = torch.cuda.current_stream(dev)
        for _ in range(warmup):
            fr()
        evs = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        seg.zero_()
        t0 = time.perf_counter()
        for _ in range(steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # the render kernel runs first in each step, on this stream: e0..e1 brackets it alone
            e0.record(stream)
            fr.render_part(fr.cfg_r, fr.part)
            e1.record(stream)
            evs.append((e0, e1))
            # rest of the step (gather + re-interleave)
            if world > 1:
                glist = list(fr.gathered.unbind(0)) if rank == 0 else None
                dist.gather(fr.part, gather_list=glist, dst=0)
            elif rank == 0:
                fr.gathered[0].copy_(fr.part)
            if rank == 0:
                rt.deinterleave_async(fr.gathered.data_ptr(), fr.world, fr.rows, W, H, fr.frame.data_ptr(),
                                      stream.cuda_stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        kern_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        t = torch.tensor([dt, kern_ms], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        segs = seg.clone()
        if world > 1:
            dist.all_reduce(segs)
        return float(t[0]), float(t[1]), [int(v) // steps for v in segs.tolist()]

    fr = make(False)
    t, kern_ms, (seg_calls, seg_traced, tri_tests, cluster_tests) = run(fr, args.steps, args.warmup)
    samples = W * H * spp
    value = samples * args.steps / t / 1e6
    frame = fr.frame.clone() if rank == 0 else None
    # per-kernel device times of the split launch (HIP events the library records around the heavy-tile
    # kernel on this stream and around the sky kernel on the scene's side stream), after the timed region:
    # reading them waits for each launch
    heavy_ms = sky_ms = None
    kt = []
    ds.set_timing(True)
    for _ in range(max(3, min(args.steps, 10))):
        fr.render_part(fr.cfg_r, fr.part)
        k = ds.kernel_times()
        if k:
            kt.append(k)
    ds.set_timing(False)
    if kt:
        heavy_ms = sum(a for a, _ in kt) / len(kt)
        sky_ms = sum(b for _, b in kt) / len(kt)
        hk = torch.tensor([heavy_ms, sky_ms], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(hk, op=dist.ReduceOp.MAX)
        heavy_ms, sky_ms = float(hk[0]), float(hk[1])

    hoisted = brute = None
    if not args.no_hoisted:
        frh = make(True)
        th, kh, (hc, ht, htests, _) = run(frh, args.steps, 1)
        hoisted = {"value": round(samples * args.steps / th / 1e6, 3), "ms_per_step": round(th / args.steps * 1e3, 4),
                   "kernel_ms": round(kh, 4), "segments_traced": ht, "tri_tests": htests,
                   "bit_exact_vs_faithful": bool(rank != 0 or torch.equal(frh.frame, frame))}
        # the same faithful frame without the tile candidate lists (every primary segment tests every
        # triangle, as calculateRayCollision does): for comparison only
        frb = make(False, tile_cull=False)
        tb, kb, (bc, bt, btests, _) = run(frb, max(2, args.steps // 2), 1)
        brute = {"value": round(samples * max(2, args.steps // 2) / tb / 1e6, 3),
                 "ms_per_step": round(tb / max(2, args.steps // 2) * 1e3, 4), "kernel_ms": round(kb, 4),
                 "tri_tests": btests, "bit_exact_vs_culled": bool(rank != 0 or torch.equal(frb.frame, frame))}

    if rank == 0:
        # D2H of the finished frame, reported separately (never `value`)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        host = frame.cpu()
        d2h_ms = (time.perf_counter() - t0) * 1e3
        T = len(tris)
        # ray-triangle tests the kernel evaluated per frame, all ranks (device counter: each traced segment x
        # the triangles it visits -- its tile's candidates for a primary segment, all T otherwise)
        tests = tri_tests
        # per launch on one GPU: this rank's share of the tests; kernel time = mean of its launches
        tests_per_launch = tests / world
        # the dominant kernel: rtc_render_heavy (every ray-triangle test runs there; the sky kernel tests none)
        dom_ms = heavy_ms if heavy_ms else kern_ms
        achieved_tf = tests_per_launch * FLOPS_PER_TEST / (dom_ms * 1e-3) / 1e12
        # SURVEY §8(d)'s brute-force count (traced segments x T x 57): the work calculateRayCollision does
        bf_tf = seg_traced / world * T * FLOPS_PER_TEST / (kern_ms * 1e-3) / 1e12
        scene_bytes = T * 68
        out_bytes = fr.rows * W * 3
        alg_bytes = scene_bytes + out_bytes
        traffic = None
        pmc_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            try:
                pm = json.load(open(pmc_path)).get(args.workload)
                if pm and pm.get("n_gpus", 1) == world:
                    traffic = pm["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
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
                       "mode": "faithful (every sample re-traces its primary ray: primary segments over the 8x8 tile's "
                            "candidate triangles, bounce segments over the triangle clusters their half-line may reach)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": FP32_VALU_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_VALU_PEAK_TFLOPS, 4),
                         "traffic": traffic,
                         "kernel": "rtc_render_heavy" if heavy_ms else "rtc_render_kernel",
                         "kernel_ms": round(dom_ms, 4),
                         "sky_kernel_ms": round(sky_ms, 4) if sky_ms else None,
                         "launch_ms": round(kern_ms, 4),
                         "work_per_launch": f"{tests_per_launch:.4g} ray-triangle tests x {FLOPS_PER_TEST} flop",
                         "cluster_tests_per_launch": cluster_tests // world,
                         "hbm_achieved_gbs": round(alg_bytes / (dom_ms * 1e-3) / 1e9, 3),
                         "hbm_peak_gbs": HBM_PEAK_GBS,
                         "bruteforce_equiv_tflops": round(bf_tf, 3),
                         # SURVEY.md §8(d)'s formula: segments_traced x T x 57 / (t x 157.3e12 x G); above 1
                         # because the culling layers skip ~99 % of the brute-force tests (bit-exactly)
                         "survey_formula_frac": round(bf_tf / FP32_VALU_PEAK_TFLOPS, 4),
                         "note": "achieved: the ray-triangle tests evaluated x 57 flop / the heavy-tile kernel's "
                                 "device time (HIP events around it); launch_ms: the whole launch sequence (cull, "
                                 "order, sky || heavy, counters); bruteforce_equiv: segments x T (the reference's "
                                 "brute-force work) over launch_ms"},
            "frame_ms": round(t / args.steps * 1e3, 4),
            "segments_per_frame": seg_calls,
            "segments_traced_per_frame": seg_traced,
            "msegments_per_s": round(seg_traced * args.steps / t / 1e6, 2),
            "tri_tests_per_frame": tests,
            "gtests_per_s": round(tests * args.steps / t / 1e9, 2),
            "d2h_ms": round(d2h_ms, 3),
            "hoisted": hoisted,
            "no_tile_cull": brute,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb, ccol = cpu_baseline(tris, tonly, scene, cam, W, H, spp, args.cpu_row_stride)
            gpu_rows = host.numpy()[::args.cpu_row_stride]
            cb["u8_mismatch_vs_gpu"] = int((gpu_rows != ccol).any(-1).sum())
            cb.pop("seconds")
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(line), flush=True)
    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""One rank's share of a frame at N GPUs (rows y = r + kN), rendered on one GPU: the per-rank device time that
bounds strong scaling (the gather of the uint8 parts and the re-interleave come on top).  Not part of the product.
Usage: scale_probe.py [frames] [W H spp] [kernel: chain|overlap|overlap_inline]  (SCALE_NS=1,8: the N to probe;
SCALE_BAND=8: bands of 8 rows instead of single rows; overlap: the chain kernel with frame
pipelining, RTC_F_OVERLAP -- the per-frame period of back-to-back frames instead of one frame's latency)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 7
W, H, SPP = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
kernel = sys.argv[5] if len(sys.argv) > 5 else "chain"
extra = {"chain": {}, "overlap": {"overlap": True}, "overlap_inline": {"overlap": True, "chain_inline": True},
         "overlap_hoist": {"overlap": True, "hoist": True}}[kernel]
NS = tuple(int(v) for v in os.environ.get("SCALE_NS", "1,2,4,8").split(","))
BAND = int(os.environ.get("SCALE_BAND", "1"))  # rows per interleaved band (rtc.h rowBand; 1: single rows)
tris, _ = load_tris("ultracomplex")
scene, cam = rt.default_scene(), rt.camera_basis()
ds = rt.DeviceScene(tris, None)
stream = torch.cuda.current_stream()
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
for _ in range(20):  # clocks settle
    ds.render_rows_async(scene, cam, rt.RenderConfig(W, H, SPP, 10, True, **extra), out.data_ptr(), None, None,
                         stream.cuda_stream)
torch.cuda.synchronize()
base = None
for n in NS:
    worst = 0.0
    per = []
    for r in range(n):  # every rank's share: the slowest sets the frame
        cfg = rt.RenderConfig(W, H, SPP, 10, True, row_start=r * BAND, row_stride=n, row_band=BAND if BAND > 1 else 0,
                              **extra)
        times = []
        if kernel.startswith("overlap"):  # the period of 20 back-to-back pipelined frames (device synchronised around them)
            for _ in range(frames):
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(20):
                    ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, stream.cuda_stream)
                torch.cuda.synchronize()
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 20)
        else:
            for _ in range(frames):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
        ms = sorted(times)[len(times) // 2]
        per.append(round(ms, 4))
        worst = max(worst, ms)
    if base is None:
        base = worst
    print(json.dumps({"n": n, "W": W, "H": H, "spp": SPP, "kernel": kernel, "band": BAND, "rank_ms": per, "slowest_ms": round(worst, 4),
                      "ideal_ms": round(base / n, 4), "speedup_bound": round(base / worst, 3),
                      "efficiency_bound": round(base / n / worst, 3)}), flush=True)
ds.close()

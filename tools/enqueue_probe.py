#!/usr/bin/env python3
"""Host cost of enqueueing pipelined launches vs the GPU period (not part of the product): for the whole 1080p frame
and rank 0's 1/4 and 1/8 shares, the wall time of each render_rows_async call (no synchronisation inside the loop) and
the device period of the same 100 launches.  Usage: enqueue_probe.py"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

tris, _ = load_tris("ultracomplex")
ds = rt.DeviceScene(tris, None)
scene, cam = rt.default_scene(), rt.camera_basis()
st = torch.cuda.current_stream()
out = torch.zeros((1080, 1920, 3), dtype=torch.uint8, device="cuda")
for n in (1, 4, 8):
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True, overlap=True, row_stride=n)
    for _ in range(20):
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
    torch.cuda.synchronize()
    per = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    t0 = time.perf_counter()
    for _ in range(100):
        a = time.perf_counter()
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
        per.append(time.perf_counter() - a)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    e1.record(st)
    torch.cuda.synchronize()
    per.sort()
    print(json.dumps({"n": n, "host_us_per_call_median": round(per[50] * 1e6, 1), "host_us_per_call_p90": round(per[90] * 1e6, 1),
                      "host_loop_us_per_frame": round(t_host / 100 * 1e6, 1),
                      "device_period_us": round(e0.elapsed_time(e1) / 100 * 1e3, 1)}), flush=True)
ds.close()

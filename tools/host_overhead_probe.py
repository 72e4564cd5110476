#!/usr/bin/env python3
"""Host cost of enqueuing one frame vs its device time, at a rank's share of the BASELINE frame for N = 1, 2, 4,
8 (rows y = r + kN on one GPU): if the host needs longer to enqueue a frame than the GPU needs to render it, a
multi-GPU step is host-bound.  Not part of the product.  Usage: host_overhead_probe.py [frames]"""
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

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H, SPP = 1920, 1080, 64
tris, _ = load_tris("ultracomplex")
scene, cam = rt.default_scene(), rt.camera_basis()
ds = rt.DeviceScene(tris, None)
stream = torch.cuda.Stream()
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
for n in (1, 2, 4, 8):
    cfg = rt.RenderConfig(W, H, SPP, 10, True, row_start=0, row_stride=n)
    for _ in range(20):
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, stream.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frames):
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, stream.cuda_stream)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(json.dumps({"n": n, "host_enqueue_us_per_frame": round(t_host / frames * 1e6, 2),
                      "device_us_per_frame": round(t_all / frames * 1e6, 2)}), flush=True)
ds.close()

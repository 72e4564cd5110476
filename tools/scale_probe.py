#!/usr/bin/env python3
"""One rank's share of the 1080p x64 ultracomplex frame at N GPUs (rows y = r + kN), rendered on one GPU:
the per-rank device time that bounds strong scaling.  Not part of the product.
Usage: scale_probe.py [frames] [lib-suffix]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 5
tris, _ = load_tris("ultracomplex")
scene, cam = rt.default_scene(), rt.camera_basis()
W, H, SPP = 1920, 1080, 64
ds = rt.DeviceScene(tris, None)
ds.set_timing(True)
stream = torch.cuda.current_stream()
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device="cuda")
base = None
for n in (1, 2, 4, 8):
    for r, lanes in [(0, 0), (0, -1)]:
        cfg = rt.RenderConfig(W, H, SPP, 10, True, row_start=r, row_stride=n, pipe=(lanes == 0))
        times, kts = [], []
        for _ in range(frames):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, seg.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
            kts.append(ds.kernel_times())
        ms = sorted(times)[len(times) // 2]
        if n == 1 and base is None:
            base = ms
        heavy = sorted(k[0] for k in kts if k)[len(kts) // 2] if any(kts) else None
        print(json.dumps({"n": n, "rank": r, "kernel": "pipe" if lanes == 0 else "coop", "ms_median": round(ms, 3), "heavy_ms": round(heavy, 3) if heavy else None,
                          "ideal_ms": round(base / n, 3), "efficiency_if_only_this": round(base / n / ms, 3)}),
              flush=True)
ds.close()

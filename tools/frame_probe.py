#!/usr/bin/env python3
"""Repeated frames on one device-resident scene (as bench.py renders them), per variant, timed with events on
the launch stream.  Not part of the product.  Usage: frame_probe.py [frames]"""
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
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
for name, t, cfg in [("empty", tris[:0], rt.RenderConfig(W, H, SPP, 10, True)),
                     ("faithful", tris, rt.RenderConfig(W, H, SPP, 10, True)),
                     ("faithful_nocluster", tris, rt.RenderConfig(W, H, SPP, 10, True, cluster_cull=False)),
                     ("faithful_nocoop", tris, rt.RenderConfig(W, H, SPP, 10, True, coop=False)),
                     ("faithful_spec", tris, rt.RenderConfig(W, H, SPP, 10, True, spec=True)),
                     ("hoist", tris, rt.RenderConfig(W, H, SPP, 10, True, hoist=True))]:
    ds = rt.DeviceScene(t, None)
    times = []
    for _ in range(frames):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, seg.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ds.close()
    print(json.dumps({"variant": name, "ms": [round(x, 3) for x in times],
                      "segments": [int(v) for v in seg.cpu()]}), flush=True)
    seg.zero_()

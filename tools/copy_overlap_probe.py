#!/usr/bin/env python3
"""Frame loop with frame k's copy (rtc_copy_async, 32 workgroups) issued at frame k+1's geometry-done event:
into pinned host memory (D2H) or into another HBM buffer (D2D), against no copy.  Does the copy slow the
concurrent sky pass because of where it writes?  Not part of the product.  Usage: copy_overlap_probe.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
W, H, SPP = 1920, 1080, 64
tris, _ = load_tris("ultracomplex")
sc, cam = rt.default_scene(), rt.camera_basis()
ds = rt.DeviceScene(tris, None, device=0)
cfg = rt.RenderConfig(W, H, SPP, 10, True)
rs, cs = torch.cuda.Stream(), torch.cuda.Stream()
geo = torch.cuda.Event()
geo.record(rs)
torch.cuda.synchronize()
ds.set_geometry_event(geo.cuda_event)
dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]
host = [torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(3)]
dev2 = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]


def loop(dst, blocks=32):
    copied = [None] * 3
    pending = None
    t0 = None
    for k in range(steps + 10):
        if k == 10:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        b = k % 3
        if copied[b] is not None:
            rs.wait_event(copied[b])
        ds.render_rows_async(sc, cam, cfg, dev[b].data_ptr(), None, None, rs.cuda_stream)
        if dst is not None:
            if pending is not None:
                cs.wait_event(geo)
                rt.copy_async(dst[pending].data_ptr(), dev[pending].data_ptr(), dev[pending].numel(), blocks,
                              cs.cuda_stream)
                e = torch.cuda.Event()
                e.record(cs)
                copied[pending] = e
            pending = b
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for rep in range(2):
    print("none", round(loop(None), 4), "d2h", round(loop(host), 4), "d2d", round(loop(dev2), 4),
          "d2h_8blocks", round(loop(host, 8), 4), flush=True)
ds.close()

#!/usr/bin/env python3
"""Frame loop with the D2H of frame k overlapping frame k+1's render, under stream-priority variants (which
stream's kernels the dispatcher prefers: the render's or the copy's blit kernel).  Not part of the product.
Usage: d2h_overlap_probe.py [steps]"""
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
lo, hi = torch.cuda.Stream.priority_range()
print("priority range (least, greatest):", lo, hi, flush=True)
dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
host = [torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(2)]


def loop(rs, cs, d2h=True):
    copied = [None, None]

    def one(k):
        b = k % 2
        if copied[b] is not None:
            rs.wait_event(copied[b])
        ds.render_rows_async(sc, cam, cfg, dev[b].data_ptr(), None, None, rs.cuda_stream)
        if d2h:
            ev = torch.cuda.Event()
            ev.record(rs)
            cs.wait_event(ev)
            with torch.cuda.stream(cs):
                host[b].copy_(dev[b], non_blocking=True)
            done = torch.cuda.Event()
            done.record(cs)
            copied[b] = done
    for k in range(10):
        one(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        one(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


variants = {
    "default_stream+copy_normal": (torch.cuda.current_stream(), torch.cuda.Stream()),
    "render_normal+copy_normal": (torch.cuda.Stream(), torch.cuda.Stream()),
    "render_high+copy_normal": (torch.cuda.Stream(priority=hi), torch.cuda.Stream()),
    "render_high+copy_least": (torch.cuda.Stream(priority=hi), torch.cuda.Stream(priority=lo)),
}
for rep in range(2):
    for name, (rs, cs) in variants.items():
        print(name, "d2h", round(loop(rs, cs), 4), "device_only", round(loop(rs, cs, False), 4), flush=True)
ds.close()

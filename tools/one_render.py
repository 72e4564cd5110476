#!/usr/bin/env python3
"""One render of a chosen variant (for rocprofv3 counter passes).  Usage: one_render.py [variant] [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

v = sys.argv[1] if len(sys.argv) > 1 else "faithful"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tris, _ = load_tris("ultracomplex")
import bench  # noqa: E402  (a bench.py workload name renders that workload)

if v in bench.WORKLOADS:
    # the bench's own launch: device-resident scene, no segment counters (the timed kernel instantiation), pipelined
    import torch

    name, W, H, spp = bench.WORKLOADS[v]
    tris, _ = load_tris(name)
    cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=True)  # launched like the bench's timed frames
    ds = rt.DeviceScene(tris, None, device=0)
    out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream()
    for _ in range(reps):
        ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, out.data_ptr(), None, None, s.cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    print(v, "rendered", reps)
    sys.exit(0)
if v in ("share4o", "share8o", "fullo"):
    # pipelined launches like tools/scale_probe.py overlap: rank 0's share of N = 4 / 8, or the whole frame
    import torch

    n = {"share4o": 4, "share8o": 8, "fullo": 1}[v]
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True, overlap=True, row_stride=n)
    ds = rt.DeviceScene(tris, None, device=0)
    out = torch.empty((1080, 1920, 3), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream()
    for _ in range(reps):
        ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, out.data_ptr(), None, None, s.cuda_stream)
    torch.cuda.synchronize()
    ds.close()
    print(v, "rendered", reps)
    sys.exit(0)
cfg = {"faithful": rt.RenderConfig(1920, 1080, 64, 10, True),
       "nocull": rt.RenderConfig(1920, 1080, 64, 10, True, tile_cull=False), "mb1": rt.RenderConfig(1920, 1080, 64, 1, True),
       "hoist": rt.RenderConfig(1920, 1080, 64, 10, True, hoist=True),
       "empty": rt.RenderConfig(1920, 1080, 64, 10, True),
       "share8": rt.RenderConfig(1920, 1080, 64, 10, True, row_stride=8),
       "fsuzane": rt.RenderConfig(1920, 1080, 64, 10, True),
       "ns4k": rt.RenderConfig(3840, 2160, 64, 10, True)}[v]
if v == "empty":
    tris = tris[:0]
if v == "fsuzane":
    tris, _ = load_tris("fsuzane")
for _ in range(reps):
    _, _, st = rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
print(v, st["render_ms"])

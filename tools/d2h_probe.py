#!/usr/bin/env python3
"""How the frame reaches host memory: timings of the variants bench.py could use (not part of the product).

  device   : render into HBM only (no D2H)
  serial   : render into HBM, hipMemcpyAsync D2H into pinned memory on the same stream
  overlap  : render into HBM, D2H on a copy stream overlapping the next frame (double-buffered)
  zerocopy : the render kernels write Color[] straight into pinned host memory (device-visible)
  copyonly : the D2H alone
Usage: d2h_probe.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H, SPP = 1920, 1080, 64
tris, _ = load_tris("ultracomplex")
scene, cam = rt.default_scene(), rt.camera_basis()
ds = rt.DeviceScene(tris, None, device=0)
cfg = rt.RenderConfig(W, H, SPP, 10, True)
st = torch.cuda.current_stream()
cs = torch.cuda.Stream()
dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
host = [torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(2)]


def render(ptr):
    ds.render_rows_async(scene, cam, cfg, ptr, None, None, st.cuda_stream)


def timed(fn):
    for k in range(3):
        fn(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


copied = [None, None]


def overlap(k):
    b = k % 2
    if copied[b] is not None:
        st.wait_event(copied[b])
    render(dev[b].data_ptr())
    ev = torch.cuda.Event()
    ev.record(st)
    cs.wait_event(ev)
    with torch.cuda.stream(cs):
        host[b].copy_(dev[b], non_blocking=True)
    done = torch.cuda.Event()
    done.record(cs)
    copied[b] = done


res = {
    "device": timed(lambda k: render(dev[k % 2].data_ptr())),
    "serial": timed(lambda k: (render(dev[0].data_ptr()), host[0].copy_(dev[0], non_blocking=True))),
    "overlap": timed(overlap),
    "zerocopy": timed(lambda k: render(host[k % 2].data_ptr())),
    "copyonly": timed(lambda k: host[k % 2].copy_(dev[k % 2], non_blocking=True)),
}
ref = dev[0].cpu()
render(host[0].data_ptr())
torch.cuda.synchronize()
res["zerocopy_equal"] = bool(torch.equal(host[0], ref))
print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()})

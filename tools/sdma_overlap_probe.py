#!/usr/bin/env python3
"""Frame loop with each frame's D2H done by the SDMA engines (HSA, tools/sdma_copy.cpp) from a host thread once
the frame is complete, against the CU copy (rtc_copy_async) and no copy.  Not part of the product."""
import ctypes as C
import os
import sys
import threading
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
rs = torch.cuda.Stream()
dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]
host = [torch.empty((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(3)]
sd = C.CDLL(os.path.join(REPO, "raytracingc_amd", "_lib", "libsdma_copy.so"))
sd.sdma_copy_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
print("sdma_init", sd.sdma_init(), flush=True)


def loop_sdma():
    done_ev = [None] * 3
    copied = [threading.Event() for _ in range(3)]
    for e in copied:
        e.set()
    jobs = []

    def worker(b, ev):
        ev.synchronize()
        sd.sdma_copy_d2h(host[b].data_ptr(), dev[b].data_ptr(), dev[b].numel())
        copied[b].set()

    t0 = time.perf_counter()
    for k in range(steps):
        b = k % 3
        copied[b].wait()
        copied[b].clear()
        ds.render_rows_async(sc, cam, cfg, dev[b].data_ptr(), None, None, rs.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(rs)
        th = threading.Thread(target=worker, args=(b, ev))
        th.start()
        jobs.append(th)
    for th in jobs:
        th.join()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def loop_none():
    t0 = time.perf_counter()
    for k in range(steps):
        ds.render_rows_async(sc, cam, cfg, dev[k % 3].data_ptr(), None, None, rs.cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for _ in range(10):
    ds.render_rows_async(sc, cam, cfg, dev[0].data_ptr(), None, None, rs.cuda_stream)
torch.cuda.synchronize()
for rep in range(3):
    print("none", round(loop_none(), 4), "sdma", round(loop_sdma(), 4), flush=True)
ref = dev[(steps - 1) % 3].cpu()
print("host equals device", bool(torch.equal(host[(steps - 1) % 3], ref)))
ds.close()

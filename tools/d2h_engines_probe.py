#!/usr/bin/env python3
"""Device-to-host copy rate of rtc_copy_d2h_dma (SDMA) for a 1080p and a 4K frame; checks the bytes.  Not part
of the product.  Usage: d2h_engines_probe.py
(r02: one engine already moves ~52-54 GB/s, the PCIe limit: 0.12 ms per 1080p frame, 0.46 ms per 4K frame;
the split over 2-4 engines measured the same and was not kept)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402

out = {}
for name, n in (("1080p", 1920 * 1080 * 3), ("4k", 3840 * 2160 * 3)):
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    for _ in range(5):
        rt.copy_d2h_dma(dst.data_ptr(), src.data_ptr(), n)
    t0 = time.perf_counter()
    reps = 40
    for _ in range(reps):
        rt.copy_d2h_dma(dst.data_ptr(), src.data_ptr(), n)
    dt = (time.perf_counter() - t0) / reps
    out[name] = {"ms": round(dt * 1e3, 4), "GBps": round(n / dt / 1e9, 1), "exact": bool(torch.equal(dst, src.cpu()))}
print(json.dumps(out), flush=True)

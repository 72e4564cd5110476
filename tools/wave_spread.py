#!/usr/bin/env python3
"""Spread of rtc_render_chain's waves within one launch (diagnostic build: per-wave start / end by s_memrealtime and
items done): joined launches of a frame or a row share, one at a time.  Not part of the product.
Usage: wave_spread.py [scene W H spp G] -- G > 1: rank 0's share of G row-interleaved ranks."""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["RTC_LIB_PATH"] = os.environ.get("RTC_DIAG_LIB") or os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402
from raytracingc_amd.distributed import rank_config, rows_per_rank  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "ultracomplex"
W, H, SPP, G = (int(v) for v in sys.argv[2:6]) if len(sys.argv) > 5 else (1920, 1080, 64, 8)
tris, _ = load_tris(scene_name)
L = rt.lib()
L.rtc_diag_wavelog.argtypes = [C.c_void_p, C.c_int, C.c_int]
ds = rt.DeviceScene(tris, None)
cfg = rank_config(rt.RenderConfig(W, H, SPP, 10, True, overlap=True), 0, G) if G > 1 else \
    rt.RenderConfig(W, H, SPP, 10, True, overlap=True)
rows = rows_per_rank(H, G) if G > 1 else H
buf = torch.zeros((rows, W, 3), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
st = torch.cuda.Stream()
for _ in range(5):
    ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
torch.cuda.synchronize()
out = np.zeros((16384, 8), np.uint64)
for rep in range(3):
    L.rtc_diag_wavelog(None, 0, 1)
    ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    n = L.rtc_diag_wavelog(out.ctypes.data, 16384, 1)
    a = out[:n][out[:n, 0] != 0].astype(np.int64)  # slots with a wave
    n = len(a)
    t0 = a[:, 0].min()
    start, end, items = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, a[:, 2]  # 100 MHz ticks -> us
    q = lambda v, p: round(float(np.percentile(v, p)), 2)  # noqa: E731
    ends = a[:, 3:8]  # the end of items 1..5 (0: not reached)
    prev = a[:, 0].copy()
    item_us = []
    for k in range(5):
        ok = ends[:, k] > 0
        item_us.append(round(float(((ends[ok, k] - prev[ok]) / 100.0).mean()), 2) if ok.any() else None)
        prev = np.where(ok, ends[:, k], prev)
    print(json.dumps({"scene": scene_name, "W": W, "H": H, "spp": SPP, "G": G, "waves": int(n), "items": int(items.sum()),
                      "span_us": round(float(end.max()), 2), "start_p50_us": q(start, 50), "start_max_us": q(start, 100),
                      "end_p10_us": q(end, 10), "end_p50_us": q(end, 50), "end_p90_us": q(end, 90),
                      "end_p99_us": q(end, 99), "items_p50": q(items, 50), "items_max": int(items.max()),
                      "busy_mean_us": round(float((end - start).mean()), 2),
                      "busy_frac_of_span": round(float((end - start).sum() / (n * end.max())), 3),
                      "item_us_1_to_5": item_us}), flush=True)
ds.close()

#!/usr/bin/env python3
"""Per-workgroup timeline of rtc_tile_cull from the diagnostic build (librtc_diag.so: wave 0 of every block stamps
s_memtime at its start, after level 1 and at its end, plain stores) for the BASELINE frame and one rank's 1/8 share:
how the kernel's span splits into dispatch spread and block durations.  Not part of the product."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["RTC_LIB_PATH"] = os.environ.get("RTC_DIAG_LIB") or os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

tris, _ = load_tris("ultracomplex")
L = rt.lib()
L.rtc_diag_set_cull_buffer.argtypes = [C.c_void_p]
ds = rt.DeviceScene(tris, None)
sc, cam = rt.default_scene(), rt.camera_basis()
st = torch.cuda.current_stream()
for stride in (1, 8):
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True, row_stride=stride)
    rows = cfg.rows()
    blocks = ((1920 + 15) // 16) * ((rows + 15) // 16)
    buf = torch.zeros(blocks * 8, dtype=torch.int64, device="cuda")
    out = torch.zeros((rows, 1920, 3), dtype=torch.uint8, device="cuda")
    for _ in range(5):
        ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
    torch.cuda.synchronize()
    L.rtc_diag_set_cull_buffer(C.c_void_p(buf.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    L.rtc_diag_set_cull_buffer(None)
    r = buf.cpu().numpy().view(np.uint64).reshape(blocks, 8).astype(np.float64)
    t0 = r[:, 0].min()
    start, l1, end, geo = r[:, 0] - t0, r[:, 1] - t0, r[:, 2] - t0, r[:, 3] > 0
    dur = end - start
    span = end.max()
    g = {"blocks": blocks, "geometry_blocks": int(geo.sum()), "span_ticks": int(span),
         "frame_ms_events": round(e0.elapsed_time(e1), 4),
         "start_ticks_p50_p90_max": [int(np.percentile(start, 50)), int(np.percentile(start, 90)), int(start.max())],
         "sky_block_ticks_mean_max": [int(dur[~geo].mean()) if (~geo).any() else 0, int(dur[~geo].max()) if (~geo).any() else 0],
         "sky_level1_ticks_mean": int((l1 - start)[~geo].mean()) if (~geo).any() else 0,
         "geo_block_ticks_mean_max": [int(dur[geo].mean()) if geo.any() else 0, int(dur[geo].max()) if geo.any() else 0],
         "geo_level1_ticks_mean": int((l1 - start)[geo].mean()) if geo.any() else 0,
         "geo_prefilter2_loop_ticks_mean": [int(r[geo, 4].mean()), int(r[geo, 5].mean())] if geo.any() else None,
         "geo_candidates_mean_max": [round(r[geo, 6].mean(), 1), int(r[geo, 6].max())] if geo.any() else None,
         "slowest_block": {"geo": bool(geo[dur.argmax()]), "start": int(start[dur.argmax()]), "dur": int(dur.max()),
                           "level1": int((l1 - start)[dur.argmax()]), "prefilter2": int(r[dur.argmax(), 4]),
                           "loop": int(r[dur.argmax(), 5]), "candidates": int(r[dur.argmax(), 6])},
         "last_end_block": {"geo": bool(geo[end.argmax()]), "start": int(start[end.argmax()]), "dur": int(dur[end.argmax()])}}
    print(json.dumps({"row_stride": stride, **g}), flush=True)
ds.close()

#!/usr/bin/env python3
"""Per-heavy-tile timing of the split launch with the diagnostic build (librtc_diag.so): for each heavy tile
{realtime start, realtime end (100 MHz), shader cycles, worker/tile}.  Not part of the product."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["RTC_LIB_PATH"] = os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

tris, _ = load_tris("ultracomplex")
scene, cam = rt.default_scene(), rt.camera_basis()
W, H, SPP = 1920, 1080, 64
tiles = ((W + 15) // 16 * 2) * ((H + 15) // 16 * 2)
buf = torch.zeros(tiles * 4, dtype=torch.int64, device="cuda")
rt.lib().rtc_diag_set_buffer.argtypes = [C.c_void_p]
rt.check(rt.lib().rtc_diag_set_buffer(C.c_void_p(buf.data_ptr())), "diag")
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
ds = rt.DeviceScene(tris, None)
ds.set_timing(True)
stream = torch.cuda.current_stream()
rt.lib().rtc_diag_sections.argtypes = [C.c_void_p, C.c_int]
sect = np.zeros(16, np.uint64)
NAMES = ["primary_trace", "cluster_tests", "gen_filter", "gen_exact", "lane_reduce", "hit_shading", "sky_miss",
         "loop_total"]
STRIDE = int(os.environ.get("DIAG_STRIDE", "1"))
for hoist in (False, True):
    cfg = rt.RenderConfig(W, H, SPP, 10, True, hoist=hoist, row_stride=STRIDE,
                          spec=os.environ.get("DIAG_SPEC", "0") == "1")
    for rep in range(2):
        buf.zero_()
        rt.check(rt.lib().rtc_diag_sections(None, 1), "sections")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, None, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
    rt.check(rt.lib().rtc_diag_sections(sect.ctypes.data_as(C.c_void_p), 0), "sections")
    tot = max(float(sect[7]), 1.0)
    print(json.dumps({"hoist": hoist, "section_share_of_loop": {n: round(float(v) / tot, 3) for n, v in zip(NAMES, sect)},
                      "samples": int(sect[8]), "non7_samples": int(sect[9]), "zero_hit_samples": int(sect[10]),
                      "pixels": int(sect[11]), "max_non7_per_pixel": int(sect[12]),
                      "spec_rounds": int(sect[13]), "spec_wave_iters": int(sect[14]), "spec_pixels": int(sect[15]),
                      "loop_cycles_per_wave": round(tot / (len(np.unique(buf.view(tiles, 4)[:, 3].cpu().numpy() >> 32)) * 4), 0)}))
    d = buf.view(tiles, 4).cpu().numpy()
    m = d[:, 1] > 0
    d = d[m]
    t0 = d[:, 0].min()
    start = (d[:, 0] - t0) / 100.0  # us (100 MHz)
    end = (d[:, 1] - t0) / 100.0
    dur = end - start
    worker = d[:, 3] >> 32
    q = lambda a, p: round(float(np.percentile(a, p)), 1)
    print(json.dumps({"hoist": hoist, "frame_ms": round(e0.elapsed_time(e1), 3), "heavy_tiles": int(m.sum()),
                      "workers_used": int(len(np.unique(worker))),
                      "tile_us_p10": q(dur, 10), "tile_us_p50": q(dur, 50), "tile_us_p90": q(dur, 90),
                      "tile_us_max": round(float(dur.max()), 1),
                      "start_us_p50": q(start, 50), "start_us_max": round(float(start.max()), 1),
                      "end_us_max": round(float(end.max()), 1),
                      "tiles_started_after_200us": int((start > 200).sum()),
                      "iters_p50": q(d[:, 2], 50), "iters_max": int(d[:, 2].max()),
                      "us_per_iter_p50": q(dur / np.maximum(d[:, 2], 1), 50),
                      "longest_tile_iters": int(d[np.argmax(dur), 2])}), flush=True)
    np.save(os.path.join(REPO, "gpurun_out", f"heavy_diag_hoist{int(hoist)}.npy"), d)
ds.close()

#!/usr/bin/env python3
"""Section cycles of rtc_tile_cull from the diagnostic build (librtc_diag.so, s_memtime stamps summed over waves) for
the BASELINE frame and one rank's 1/8 share.  Not part of the product.  Usage: cull_sections.py"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["RTC_LIB_PATH"] = os.environ.get("RTC_DIAG_LIB") or os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")
import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

tris, _ = load_tris("ultracomplex")
L = rt.lib()
L.rtc_diag_cull.argtypes = [C.c_void_p, C.c_int]
out = (C.c_ulonglong * 12)()
names = ["start_to_level1", "sky_block_tail", "level2_prefilter", "pixel_loops", "append_tail", "sky_waves", "geo_waves",
         "candidates_looped", "geo_level1_to_loops_done", "geo_whole"]
for stride in (1, 8):
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True, row_stride=stride)
    rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
    L.rtc_diag_cull(out, 1)
    _, _, st = rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
    L.rtc_diag_cull(out, 1)
    v = {n: int(out[i]) for i, n in enumerate(names)}
    sw, gw = max(1, v["sky_waves"]), max(1, v["geo_waves"])
    print(json.dumps({"row_stride": stride, "totals": v,
                      "per_sky_wave": {"start_to_level1": round(v["start_to_level1"] / (sw + gw)), "tail": round(v["sky_block_tail"] / sw)},
                      "per_geo_wave": {k: round(v[k] / gw) for k in ("level2_prefilter", "pixel_loops", "append_tail",
                                                                      "candidates_looped", "geo_level1_to_loops_done", "geo_whole")}}),
          flush=True)

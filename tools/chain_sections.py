#!/usr/bin/env python3
"""Section cycles of rtc_render_chain from the diagnostic build (librtc_diag.so, s_memtime stamps summed over
waves), on the BASELINE frame (or another scene: chain_sections.py fsuzane).  Not part of the product."""
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

scene_name = sys.argv[1] if len(sys.argv) > 1 else "ultracomplex"
tris, _ = load_tris(scene_name)
L = rt.lib()
L.rtc_diag_sections.argtypes = [C.c_void_p, C.c_int]
out = (C.c_ulonglong * 16)()
names = ["rng_setup", "primary_trace", "hit_shading", "cluster_cull", "pair_build", "pair_passes", "env", "walk"]
for hoist in (False, True):
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True, hoist=hoist)
    rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
    L.rtc_diag_sections(out, 1)
    _, _, st = rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
    L.rtc_diag_sections(out, 1)
    tot = sum(out[i] for i in range(8))
    it, alive, act, win, used = (out[i] for i in range(8, 13))
    print(json.dumps({"hoist": hoist, "iterations": it, "lane_utilisation": round(alive / max(1, 64 * it), 4),
                      "window_lanes_per_window": round(act / max(1, win), 2), "used_lanes_share": round(used / max(1, act), 4),
                      "iterations_per_window": round(it / max(1, win), 2)}), flush=True)
    print(json.dumps({"hoist": hoist, "render_ms": round(st["render_ms"], 3),
                      "share": {n: round(out[i] / tot, 4) for i, n in enumerate(names)},
                      "cycles": {n: int(out[i]) for i, n in enumerate(names)},
                      # 13: whole wave lifetime, 14: first-bounce tables (cluster terms, reach), 15: item fetch and
                      # pixel setup -- the sections above cover tot / lifetime of the waves' cycles
                      "wave_cycles": int(out[13]), "table_build": int(out[14]), "item_setup": int(out[15]),
                      "covered": round((tot + out[14] + out[15]) / max(1, out[13]), 4)}), flush=True)

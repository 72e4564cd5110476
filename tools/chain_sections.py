#!/usr/bin/env python3
"""Section cycles of rtc_render_chain from the diagnostic build (librtc_diag.so, s_memtime stamps summed over
waves), on the BASELINE frame (or another scene: chain_sections.py fsuzane).  Not part of the product.

Round 5: the top-level sections are uniform marks that tile each wave's lifetime (DMARK: every cycle from the kernel's
first mark to its last lands in exactly one of them, so `covered` is ~1 by construction); the finer sections nest
inside them (BEGIN/END pairs): the first-bounce table, cluster cull, pair build and pair passes inside the bounce
trace, the hit branch and the environment inside the shading."""
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

NS = 24
TOP = {19: "prologue", 15: "item_setup", 0: "window_setup", 1: "primary_trace", 17: "bounce_trace", 16: "shading",
       20: "later_bounce_trace", 21: "later_shading", 7: "walk_and_sums", 18: "item_tail"}
NESTED = {14: ("bounce_trace", "first_bounce_table"), 3: ("*bounce_trace", "cluster_cull"),
          4: ("*bounce_trace", "pair_build"), 5: ("*bounce_trace", "pair_passes"), 2: ("*shading", "hit"),
          6: ("*shading", "environment")}
scene_name = sys.argv[1] if len(sys.argv) > 1 else "ultracomplex"
W, H, SPP = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
tris, _ = load_tris(scene_name)
L = rt.lib()
L.rtc_diag_sections.argtypes = [C.c_void_p, C.c_int]
out = (C.c_ulonglong * NS)()
for hoist in (False, True):
    # pipelined launches like the bench's timed frames (in-kernel sums on the alternating streams), one at a time
    import torch

    cfg = rt.RenderConfig(W, H, SPP, 10, True, hoist=hoist, overlap=True)
    ds = rt.DeviceScene(tris, None)
    buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    for _ in range(3):
        ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    L.rtc_diag_sections(out, 1)
    ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    L.rtc_diag_sections(out, 1)
    ds.close()
    life = out[13]
    top = {n: int(out[i]) for i, n in TOP.items()}
    nested = {f"{p}/{n}": int(out[i]) for i, (p, n) in NESTED.items()}
    it, alive, act, win, used = (out[i] for i in range(8, 13))
    print(json.dumps({"scene": scene_name, "W": W, "H": H, "spp": SPP, "hoist": hoist, "iterations": it,
                      "lane_utilisation": round(alive / max(1, 64 * it), 4),
                      "window_lanes_per_window": round(act / max(1, win), 2),
                      "used_lanes_share": round(used / max(1, act), 4),
                      "iterations_per_window": round(it / max(1, win), 2),
                      "later_iterations": int(out[22]),
                      "later_lane_utilisation": round(out[23] / max(1, 64 * out[22]), 4)}), flush=True)
    print(json.dumps({"hoist": hoist, "wave_cycles": int(life),
                      "share": {n: round(v / max(1, life), 4) for n, v in top.items()},
                      "nested_share": {n: round(v / max(1, life), 4) for n, v in nested.items()},
                      "cycles": top, "nested_cycles": nested,
                      "covered": round(sum(top.values()) / max(1, life), 4)}), flush=True)

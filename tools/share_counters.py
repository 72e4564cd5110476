#!/usr/bin/env python3
"""Work counters of one rank's share (rows y = r + kN) against the whole frame: segments, ray-triangle tests
(primary + bounce), geometry items -- where a small interleaved share spends more per pixel than the frame does.
Not part of the product.  Usage: share_counters.py [W H spp]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

W, H, SPP = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (1920, 1080, 64)
tris, _ = load_tris("ultracomplex")
BAND = int(os.environ.get("SCALE_BAND", "1"))  # rows per interleaved band (1: single rows)
for n in (1, 2, 4, 8):
    for hoist in (False, True):
        # every rank's share: the per-rank balance (segments are the cost proxy, SURVEY §8 e)
        per = []
        for r in range(n):
            cfg = rt.RenderConfig(W, H, SPP, 10, True, row_start=r * BAND, row_stride=n, hoist=hoist,
                                  row_band=BAND if BAND > 1 else 0)
            _, _, st = rt.render(tris, None, rt.default_scene(), rt.camera_basis(), cfg)
            per.append(st)
        st = per[0]
        segs = [p["segments"] for p in per]
        print(json.dumps({"n": n, "band": BAND, "hoist": hoist, "rows": cfg.rows(),
                          "segments_max_over_mean": round(max(segs) * n / max(1, sum(segs)), 4),
                          "tests_max_over_mean": round(max(p["tri_tests"] for p in per) * n /
                                                       max(1, sum(p["tri_tests"] for p in per)), 4),
                          "segments": st["segments"],
                          "tri_tests": st["tri_tests"], "samples": st["samples"],
                          "tests_per_sample": round(st["tri_tests"] / max(1, st["samples"]), 4),
                          "render_ms": round(st["render_ms"], 4)}), flush=True)

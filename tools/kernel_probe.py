#!/usr/bin/env python3
"""Kernel experiments on the GPU box: time render variants, and (with the diagnostic build) the per-wave
cycle distribution.  Not part of the product; prints one JSON object per experiment."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
DIAG = "--diag" in sys.argv
if DIAG:
    os.environ["RTC_LIB_PATH"] = os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402


def timed(tris, cfg, reps=3, spheres=None):
    best = None
    for _ in range(reps):
        _, _, st = rt.render(tris, spheres, scene, cam, cfg)
        best = st if best is None or st["render_ms"] < best["render_ms"] else best
    return best


scene, cam = rt.default_scene(), rt.camera_basis()
tris, _ = load_tris(sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "ultracomplex")
W, H, SPP = 1920, 1080, 64
QUICK = "--quick" in sys.argv
if not DIAG:
    variants = {
        "faithful": (tris, rt.RenderConfig(W, H, SPP, 10, True)),
        "faithful_nocull": (tris, rt.RenderConfig(W, H, SPP, 10, True, tile_cull=False)),
        "faithful_raster": (tris, rt.RenderConfig(W, H, SPP, 10, True, reorder=False)),
        "faithful_nocoop": (tris, rt.RenderConfig(W, H, SPP, 10, True, coop=False)),
        "hoist": (tris, rt.RenderConfig(W, H, SPP, 10, True, hoist=True)),
        "mb1": (tris, rt.RenderConfig(W, H, SPP, 1, True)),
        "mb1_hoist": (tris, rt.RenderConfig(W, H, SPP, 1, True, hoist=True)),
        "empty_scene": (tris[:0], rt.RenderConfig(W, H, SPP, 10, True)),
        "one_tri": (tris[:1], rt.RenderConfig(W, H, SPP, 10, True)),
        "spp1": (tris, rt.RenderConfig(W, H, 1, 10, True)),
        "spp16": (tris, rt.RenderConfig(W, H, 16, 10, True)),
    }
    if QUICK:
        variants = {k: variants[k] for k in ("faithful", "faithful_nocull", "faithful_raster", "faithful_nocoop", "hoist", "mb1", "empty_scene")}
    for k, (t, cfg) in variants.items():
        st = timed(t, cfg)
        print(json.dumps({"variant": k, "T": len(t), "ms": round(st["render_ms"], 3), "segments": st["segments"], "tri_tests": st["tri_tests"],
                          "mrays": round(st["samples"] / st["render_ms"] / 1e3, 1)}), flush=True)
else:
    for hoist, reorder in ((False, True), (False, False), (True, True)):
        cfg = rt.RenderConfig(W, H, SPP, 10, True, hoist=hoist, reorder=reorder)
        nw = ((W + 15) // 16) * ((H + 15) // 16) * 4
        buf = torch.zeros(nw * 4, dtype=torch.int64, device="cuda")
        rt.lib().rtc_diag_set_buffer.argtypes = [C.c_void_p]
        rt.check(rt.lib().rtc_diag_set_buffer(C.c_void_p(buf.data_ptr())), "diag")
        _, _, st = rt.render(tris, None, scene, cam, cfg)
        torch.cuda.synchronize()
        d = buf.view(nw, 4).cpu().numpy()
        cyc, it, t0 = d[:, 0].astype(np.float64), d[:, 1], d[:, 2]
        span = (t0 + d[:, 0]).max() - t0.min()
        q = lambda a, p: float(np.percentile(a, p))
        print(json.dumps({"hoist": hoist, "reorder": reorder, "kernel_ms": round(st["render_ms"], 3), "waves": nw,
                          "cycles_p50": q(cyc, 50), "cycles_p90": q(cyc, 90), "cycles_p99": q(cyc, 99),
                          "cycles_max": float(cyc.max()), "cycles_sum": float(cyc.sum()),
                          "iters_p50": q(it, 50), "iters_p99": q(it, 99), "iters_max": int(it.max()),
                          "memtime_span": float(span),
                          "share_waves_over_2x_median": float((cyc > 2 * np.median(cyc)).mean()),
                          "cycles_in_waves_over_2x_median": float(cyc[cyc > 2 * np.median(cyc)].sum() / cyc.sum()),
                          "heavy_waves": int((it > 0).sum()),
                          "heavy_trace_share": float(d[it > 0, 3].sum() / max(1.0, cyc[it > 0].sum())),
                          "heavy_cycles_per_iter_p50": float(np.median(cyc[it > 0] / np.maximum(it[it > 0], 1))),
                          }), flush=True)
        np.save(os.path.join(REPO, "gpurun_out", f"wavecycles_hoist{int(hoist)}_reorder{int(reorder)}.npy"), d)

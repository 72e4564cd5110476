#!/usr/bin/env python3
"""Kernel times of one row share launched alone (joined, timing events on): the geometry kernel and the sky pass of
rank 0's share of G, against the whole frame -- how much of a pipelined share's period is its own kernels' time.
Not part of the product.  Usage: share_kernel_times.py [scene W H spp]"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402
from raytracingc_amd.distributed import rank_config, rows_per_rank  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "ultracomplex"
W, H, SPP = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
tris, _ = load_tris(scene_name)
ds = rt.DeviceScene(tris, None)
ds.set_timing(True)
st = torch.cuda.Stream()
for G in (1, 2, 4, 8):
    cfg = rank_config(rt.RenderConfig(W, H, SPP, 10, True), 0, G) if G > 1 else rt.RenderConfig(W, H, SPP, 10, True)
    buf = torch.zeros((rows_per_rank(H, G) if G > 1 else H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    kt = []
    for i in range(25):
        ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        if i >= 5:
            kt.append(ds.kernel_times())
    chain = statistics.median(k[0] for k in kt)
    sky = statistics.median(k[1] for k in kt)
    print(json.dumps({"scene": scene_name, "G": G, "chain_ms": round(chain, 4), "sky_ms": round(sky, 4)}), flush=True)
ds.close()

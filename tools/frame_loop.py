#!/usr/bin/env python3
"""Back-to-back device-resident frames of the BASELINE workload (no D2H), for rocprofv3 kernel traces of the
launch sequence and its gaps.  Not part of the product.  Usage: frame_loop.py [frames] [hoist|overlap] [row_stride] [spp]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 30
hoist = len(sys.argv) > 2 and sys.argv[2] == "hoist"
overlap = len(sys.argv) > 2 and sys.argv[2] == "overlap"
tris, _ = load_tris("ultracomplex")
ds = rt.DeviceScene(tris, None)
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # a rank's share of an N-GPU frame
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 64
cfg = rt.RenderConfig(1920, 1080, spp, 10, True, hoist=hoist, overlap=overlap, row_stride=stride)
out = torch.zeros((1080, 1920, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
sc, cam = rt.default_scene(), rt.camera_basis()
for _ in range(frames):
    ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
torch.cuda.synchronize()
print("frames", frames)

#!/usr/bin/env python3
"""Repeat the pipelined 1/G row shares of the 1080p x64 frame (tests/test_gpu_parity.py test_small_shares_sum_in_kernel)
many times in one process and report every mismatch against the joined single-GPU frame: which launch, rank, rows,
columns and whether the pixel is a geometry or a sky pixel.  A check for ordering races between consecutive overlapped
launches.  Usage: share_repeat.py [reps G band]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris, setup_from_flags  # noqa: E402
from raytracingc_amd.distributed import band_rows, rank_config, rows_per_rank  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
band = int(sys.argv[3]) if len(sys.argv) > 3 else 8
tris, _ = load_tris("ultracomplex")
scene, cam, _ = setup_from_flags({})
W, H = 1920, 1080
ref, _, _ = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, 64, 10, True), want_accum=True)
# geometry pixels, approximately: those whose colour differs from the frame of the empty scene
sky, _, _ = rt.render(tris[:0], None, scene, cam, rt.RenderConfig(W, H, 64, 10, True), want_accum=True)
geo = np.any(ref != sky, axis=2)
bad_total = 0
for rep in range(reps):
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.current_stream().cuda_stream
    rows = rows_per_rank(H, G, band)
    out = torch.zeros((G, rows, W, 3), dtype=torch.uint8, device="cuda")
    acc = torch.zeros((G, rows, W, 3), dtype=torch.float32, device="cuda")
    for r in range(G):
        cfg = rank_config(rt.RenderConfig(W, H, 64, 10, True, overlap=True), r, G, band)
        ds.render_rows_async(scene, cam, cfg, out[r].data_ptr(), acc[r].data_ptr(), None, st)
    torch.cuda.synchronize()
    ds.close()
    o = out.cpu().numpy()
    for r in range(G):
        ys = np.asarray(band_rows(H, r, G, band))
        d = np.any(o[r, :len(ys)] != ref[ys], axis=2)
        if d.any():
            rr, xx = np.nonzero(d)
            bad_total += 1
            print(json.dumps({"rep": rep, "rank": r, "pixels": int(d.sum()), "rows": sorted(set(int(ys[v]) for v in rr))[:20],
                              "x_range": [int(xx.min()), int(xx.max())], "geometry_pixels": int(geo[ys[rr], xx].sum()),
                              "sample": [[int(ys[rr[k]]), int(xx[k]), o[r, rr[k], xx[k]].tolist(),
                                          ref[ys[rr[k]], xx[k]].tolist()] for k in range(min(4, len(rr)))]}),
                  flush=True)
print(json.dumps({"reps": reps, "G": G, "band": band, "bad_rank_frames": bad_total}), flush=True)

#!/usr/bin/env python3
"""A/B timing of library variants on the BASELINE frame (not part of the product).
Usage: ab_frame.py [--frames N] [--cfg k=v ...] lib1.so lib2.so ...   (paths under raytracingc_amd/_lib/)
Each variant runs in its own process (RTC_LIB_PATH); prints the median device frame time and kernel times."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, statistics, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
import torch
import raytracingc_amd as rt
from conftest import load_tris
cfgkw = json.loads(os.environ.get("AB_CFG", "{}"))
scene_name = cfgkw.pop("scene", "ultracomplex")
W, H, SPP = cfgkw.pop("W", 1920), cfgkw.pop("H", 1080), cfgkw.pop("spp", 64)
tris, _ = load_tris(scene_name)
if cfgkw.pop("empty", False):  # every pixel sky: the sky kernel alone
    tris = tris[:0]
ds = rt.DeviceScene(tris, None)
cfg = rt.RenderConfig(W, H, SPP, 10, True, **cfgkw)
out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
sc, cam = rt.default_scene(), rt.camera_basis()
for _ in range(30):
    ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
torch.cuda.synchronize()
fr, kt = [], []
for _ in range(int(os.environ.get("AB_FRAMES", "20"))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
    e1.record(st)
    e1.synchronize()
    fr.append(e0.elapsed_time(e1))
ds.set_timing(True)
for _ in range(10):
    ds.render_rows_async(sc, cam, cfg, out.data_ptr(), None, None, st.cuda_stream)
    kt.append(ds.kernel_times())
print(json.dumps({"frame_ms": round(statistics.median(fr), 4), "heavy_ms": round(statistics.median(k[0] for k in kt if k), 4),
                  "sky_ms": round(statistics.median(k[1] for k in kt if k), 4)}))
'''
args = sys.argv[1:]
frames, cfg = "20", {}
while args and args[0].startswith("--"):
    if args[0] == "--frames":
        frames = args[1]
        args = args[2:]
    elif args[0] == "--cfg":
        k, v = args[1].split("=", 1)
        try:
            cfg[k] = json.loads(v)
        except json.JSONDecodeError:
            cfg[k] = v  # a bare string (scene=fsuzane)
        args = args[2:]
for lib in args:
    env = dict(os.environ, REPO=REPO, AB_FRAMES=frames, AB_CFG=json.dumps(cfg),
               RTC_LIB_PATH=os.path.join(REPO, "raytracingc_amd", "_lib", lib))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print(lib, r.stdout.strip() if r.returncode == 0 else ("FAILED " + r.stderr[-800:]), flush=True)

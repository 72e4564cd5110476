#!/usr/bin/env python3
"""Rows of tests/golden/kat_env_edge.npz where the device environment differs from the reference's (debug aid)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import raytracingc_amd as rt  # noqa: E402

k = np.load(os.path.join(REPO, "tests/golden", (sys.argv[1] if len(sys.argv) > 1 else "kat_env_edge") + ".npz"))
out = rt.getEnvironmentLight(k["rays"], k["scenes"])
ref = k["out"]
bad = np.where(((out.view(np.uint32) != ref.view(np.uint32)) & ~(np.isnan(out) & np.isnan(ref))).any(1))[0]
print(os.environ.get("RTC_LIB_PATH", "librtc.so"), "mismatching rows:", len(bad))
for i in bad[:25]:
    r, s = k["rays"][i], k["scenes"][i]
    print(i, "dir", [float(r["dir"][c]) for c in "xyz"], "sun", [float(s["normalizedSunDirection"][c]) for c in "xyz"],
          "focus", float(s["sunFocus"]), "I", float(s["sunIntensity"]), "ground", [float(s["groundColor"][c]) for c in "xyz"],
          "got", out[i].tolist(), "ref", ref[i].tolist())

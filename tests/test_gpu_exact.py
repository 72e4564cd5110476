"""Exhaustive GPU check of the exact f32 shortcuts of rtc_device.h (tools/exact_probe.hip, built by `make`):
sqrt_cr == the reference's sqrt-in-double rounded to float, and rcp_cr == the IEEE f32 divide 1.f / x, for
all 2^32 float bit patterns; the environment's branch-free powf == the glibc restatement for every x with the
sign bit clear at 8 exponents; the environment's smoothsteps with the constant divides == the IEEE divide for
all 2^32 inputs; the certified fast Box-Muller path == the exact restatement wherever it certifies (every float u
in (0, 1], every float theta in [0, 2 pi] at 4 rho); the sky term's main-path powf == glibc's on every normal x in
[2^-126, 1]; on the device that runs them."""
from __future__ import annotations

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

PROBE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracingc_amd", "_lib",
                     "exact_probe")


def test_exact_f32_shortcuts_all_inputs(gpu_available):
    assert os.path.exists(PROBE), "exact_probe not built (make)"
    r = subprocess.run([PROBE], capture_output=True, text=True, timeout=100)
    print(r.stdout)
    lines = [ln for ln in r.stdout.splitlines() if "mismatches" in ln]
    assert len(lines) == 7, r.stdout + r.stderr
    for ln in lines:
        assert ln.split()[2] == "0", ln
    assert r.returncode == 0

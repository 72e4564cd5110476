"""The C ABI library: loads, exports every symbol include/rtc.h declares, keeps the reference layouts, and
fails loudly (no CPU fallback) where no GPU is visible."""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO, load_tris

import raytracingc_amd as rt
from raytracingc_amd import _abi


def declared_symbols():
    txt = open(os.path.join(REPO, "include", "rtc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rtc_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = rt.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"librtc.so does not export {s}"
    assert sorted(_abi.EXPORTS) == syms


def test_library_has_gfx950_code_object():
    blob = open(rt.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts():
    assert C.sizeof(_abi.Triangle) == 68 and C.sizeof(_abi.Sphere) == 36 and C.sizeof(_abi.Scene) == 56
    assert C.sizeof(_abi.Ray) == 24 and C.sizeof(_abi.Material) == 20 and C.sizeof(_abi.Vec3) == 12
    assert C.sizeof(_abi.RtcCamera) == 52 and C.sizeof(_abi.RtcRenderDesc) == 36  # + rowBand (round 5)


def test_version_and_rows_selected():
    assert b"gfx950" in rt.lib().rtc_version()
    for h, start, stride, want in [(1080, 0, 1, 1080), (1080, 3, 8, 135), (1080, 7, 8, 135), (1079, 7, 8, 134), (5, 4, 8, 1),
                                   (5, 5, 8, 0), (0, 0, 1, 0), (10, 0, 0, 0)]:
        assert rt.RenderConfig(width=4, height=h, row_start=start, row_stride=stride).rows() == want


def test_no_gpu_fails_loudly():
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    tris, tonly = load_tris("simplest")
    with pytest.raises(rt.RtcError) as ei:
        rt.render(tris, None, rt.default_scene(), rt.camera_basis(), rt.RenderConfig(8, 8, 1))
    assert ei.value.code == _abi.RTC_ENODEV
    with pytest.raises(rt.RtcError):
        rt.rayTriangle(np.zeros(1, rt.RAY_DT), tris[:1])


def test_bad_arguments_rejected():
    L = rt.lib()
    d = _abi.RtcRenderDesc(16, 16, 1, 10, 1, 0, 1, 0)
    # null scene pointer etc. are argument errors, whatever the device state
    assert L.rtc_render(None, 0, None, 0, None, None, C.byref(d), 0, None, None, None) == _abi.RTC_EINVAL
    assert L.rtc_deinterleave_async(None, 0, 0, 0, 0, None, None) == _abi.RTC_EINVAL
    assert L.rtc_write_bmp(b"/nonexistent/dir/x.bmp", 1, 1, None) == _abi.RTC_EINVAL
    assert b"rtc_" in L.rtc_last_error() or len(L.rtc_last_error()) > 0


def test_flag_constants_match_header():
    """Every RTC_F_* / RTC_E* / RTC_SEGMENT_COUNTERS value in include/rtc.h equals the ctypes mirror's."""
    import re

    import raytracingc_amd._abi as abi

    txt = open(os.path.join(REPO, "include", "rtc.h")).read()
    found = dict(re.findall(r"#define\s+(RTC_(?:F_\w+|E\w+|OK|SEGMENT_COUNTERS))\s+\(?(-?(?:0x)?[0-9a-fA-F]+)\)?", txt))
    assert "RTC_F_OVERLAP" in found and "RTC_F_CHAIN_INLINE" in found
    for name, val in found.items():
        if hasattr(abi, name):
            assert getattr(abi, name) == int(val, 0), name
    for name in [n for n in found if n.startswith("RTC_F_")]:
        assert hasattr(abi, name), f"{name} missing from raytracingc_amd/_abi.py"


def test_dma_timeout_bookkeeping():
    """an SDMA copy that times out may still write its destination.  The library lists it (here a
    simulated one, rtc_dma_debug_inflight: no copy engine needed) until it ends: rtc_dma_pending counts the listed
    copies overlapping a range, rtc_host_unregister refuses such a range with RTC_EBUSY, and the entry is dropped once
    the copy is known to have ended (include/rtc.h, RTC_ETIMEDOUT contract)."""
    L = rt.lib()
    buf = (C.c_ubyte * 4096)()
    p = C.addressof(buf)
    assert rt.dma_pending(p, 4096) == 0
    assert L.rtc_dma_debug_inflight(C.c_void_p(p + 1024), 512, 1) == 0
    try:
        assert rt.dma_pending(p, 4096) == 1
        assert rt.dma_pending(p, 1024) == 0  # [p, p + 1024) ends where the copy's range starts
        assert rt.dma_pending(p + 1535, 1) == 1 and rt.dma_pending(p + 1536, 64) == 0
        assert rt.dma_pending(None) >= 1
        assert L.rtc_host_unregister(C.c_void_p(p + 1024)) == _abi.RTC_EBUSY
        assert b"timed-out" in L.rtc_last_error()
        with pytest.raises(rt.RtcError) as ei:
            rt.host_unregister(p + 1024)
        assert ei.value.code == _abi.RTC_EBUSY
    finally:
        assert L.rtc_dma_debug_inflight(C.c_void_p(p + 1024), 512, 0) == 0
    assert rt.dma_pending(p, 4096) == 0
    # dropping a copy that is not listed, or an empty range, is an argument error
    assert L.rtc_dma_debug_inflight(C.c_void_p(p), 512, 0) == _abi.RTC_EINVAL
    assert L.rtc_dma_debug_inflight(None, 0, 1) == _abi.RTC_EINVAL
    assert L.rtc_dma_pending(None, 16) == _abi.RTC_EINVAL


def test_bench_orbit_cameras():
    """bench.py's moving-camera leg: distinct origins at the default camera's distance and height, all looking at
    the default point (main.c:252-255 bases), the middle of the sweep near the default camera."""
    import math
    import sys

    sys.path.insert(0, REPO)
    import bench

    cams = bench.orbit_cameras(rt)
    assert len(cams) == bench.ORBIT_FRAMES
    origins = {(c.origin.x, c.origin.y, c.origin.z) for c in cams}
    assert len(origins) == len(cams)
    lx, ly, lz = rt.DEFAULT_LOOKING_AT
    ox, oy, oz = rt.DEFAULT_ORIGIN
    r0 = math.hypot(ox - lx, oz - lz)
    for c in cams:
        assert abs(c.origin.y - oy) < 1e-6 and abs(math.hypot(c.origin.x - lx, c.origin.z - lz) - r0) < 1e-4
        # ez is the unit vector towards the look-at point
        d = (lx - c.origin.x, ly - c.origin.y, lz - c.origin.z)
        n = math.sqrt(sum(v * v for v in d))
        assert abs(c.ez.x - d[0] / n) < 1e-5 and abs(c.ez.z - d[2] / n) < 1e-5


def test_ctypes_signatures_match_header():
    """Every argtypes list of the ctypes mirror has as many entries as the header's prototype has parameters."""
    txt = open(os.path.join(REPO, "include", "rtc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    L = rt.lib()
    checked = 0
    for name, params in re.findall(r"\b(rtc_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", txt):
        params = params.strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        at = getattr(L, name).argtypes
        if at is not None:
            assert len(at) == n, f"{name}: {len(at)} argtypes, header declares {n} parameters"
            checked += 1
    assert checked >= 25


@pytest.mark.parametrize("switch", ["RTC_AB_CHEAP_DIR", "RTC_AB_CHEAP_ENV_SKY", "RTC_AB_NO_SLOTS"])
def test_experiment_switches_need_rtc_experiment(switch):
    """the RTC_AB_* timing switches change the frame, so the device sources refuse to compile with one
    unless RTC_EXPERIMENT is defined too (the Makefile's product targets never define it)."""
    import shutil
    import subprocess

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    src = os.path.join(REPO, "raytracingc_amd", "csrc", "rtc_render.hip")
    base = [hipcc, "--offload-arch=gfx950", "-std=c++17", "-E", src, "-o", os.devnull]
    bad = subprocess.run(base + ["-D" + switch], capture_output=True, text=True, timeout=300)
    assert bad.returncode != 0 and "RTC_EXPERIMENT" in bad.stderr
    ok = subprocess.run(base + ["-D" + switch, "-DRTC_EXPERIMENT"], capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stderr[-500:]
    assert "RTC_EXPERIMENT" not in open(os.path.join(REPO, "Makefile")).read()

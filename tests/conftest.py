"""Shared test helpers.  `-m gpu` tests need an MI355X; everything else runs on the CPU container.

Scenes come from tests/golden/scenes/*.tris: the Triangle[] the reference's own loaders produced
(tests/golden/make_golden.py), so no test here reads /root/reference except the loader tests, which skip
when it is absent (it never exists on the GPU box).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
REFERENCE = os.environ.get("RTC_REFERENCE", "/root/reference")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from raytracingc_amd._abi import SPHERE_DT, TRIANGLE_DT  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


def load_tris(name: str):
    """(Triangle[] as TRIANGLE_DT, trianglesOnly) for a golden scene."""
    raw = open(os.path.join(GOLDEN, "scenes", name + ".tris"), "rb").read()
    count, tonly = np.frombuffer(raw[:8], np.int32)
    tris = np.frombuffer(raw[8:8 + 68 * int(count)], TRIANGLE_DT).copy()
    return tris, int(tonly)


def scene_spheres(name: str):
    """Spheres of a scene: the default mode has scene.h's sphere, OBJ mode none (main.c:241)."""
    if name == "default":
        s = np.zeros(1, SPHERE_DT)
        s["pos"]["y"] = 1
        s["r"] = 2.5
        s["mat"]["color"]["x"] = s["mat"]["color"]["y"] = s["mat"]["color"]["z"] = 1
        return s
    return np.zeros(0, SPHERE_DT)


def render_golden():
    with open(os.path.join(GOLDEN, "render_golden.json")) as f:
        return json.load(f)


def setup_from_flags(flags: dict):
    """(Scene, RtcCamera, maxBounce) for a golden render configuration's reference CLI flags."""
    import raytracingc_amd as rt

    scene = rt.default_scene(sun=flags.get("sun", rt.DEFAULT_SUN), ground=flags.get("ground"),
                             horizon=flags.get("horizon"), zenith=flags.get("zenith"), focus=flags.get("focus"),
                             intensity=flags.get("intensity"))
    cam = rt.camera_basis(flags.get("origin", rt.DEFAULT_ORIGIN), flags.get("looking_at", rt.DEFAULT_LOOKING_AT),
                          flags.get("fov", rt.DEFAULT_FOV))
    return scene, cam, flags.get("max_bounce", 10)


def have_ref_binary() -> bool:
    return os.path.exists(os.path.join(REPO, "oracle", "_ref", "rtc_ref"))


@pytest.fixture(scope="session")
def gpu_available():
    import raytracingc_amd as rt

    if rt.device_count() <= 0:
        pytest.fail("no GPU visible to librtc.so (the -m gpu tests must run on the MI355X box)")
    return True

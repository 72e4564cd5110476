"""The CPU oracle (oracle/rtc_oracle.c) pinned against the reference's own outputs (tests/golden/, produced by
oracle/_ref/rtc_ref = the reference sources built by `make ref`).  Everything here is bit-exact."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from conftest import GOLDEN, load_tris, render_golden, scene_spheres, setup_from_flags

import oracle.binding as orc
from raytracingc_amd._abi import RtcRenderDesc


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_rng_kat():
    k = np.load(f"{GOLDEN}/kat_rng.npz")
    u, g, d = orc.random_sequences(k["seeds"], k["uniform"].shape[1])
    assert np.array_equal(_bits(u), _bits(k["uniform"]))
    assert np.array_equal(_bits(g), _bits(k["normal"]))
    assert np.array_equal(_bits(d), _bits(k["direction"]))


def test_rng_known_answer_seed0():
    # seed 0 -> 0.0302, 0.1356, 0.2342, 0.3406
    u, _, _ = orc.random_sequences(np.array([0], np.uint32), 4)
    assert np.allclose(u[0], [0.0302, 0.1356, 0.2342, 0.3406], atol=5e-5)


def test_ray_triangle_kat():
    k = np.load(f"{GOLDEN}/kat_tri.npz")
    hit, dst = orc.ray_triangle(k["rays"], k["tris"])
    assert np.array_equal(hit, k["didHit"])
    m = hit == 1
    assert np.array_equal(_bits(dst[m]), _bits(k["dst"][m]))
    assert 0.05 < m.mean() < 0.95  # the KAT exercises both outcomes


def test_ray_sphere_kat():
    k = np.load(f"{GOLDEN}/kat_sphere.npz")
    hit, dst, nrm = orc.ray_sphere(k["rays"], k["spheres"])
    assert np.array_equal(hit, k["didHit"])
    m = hit == 1
    assert np.array_equal(_bits(dst[m]), _bits(k["dst"][m]))
    assert np.array_equal(_bits(nrm[m]), _bits(k["normal"][m]))


@pytest.mark.parametrize("fixture", ["kat_env", "kat_env_edge"])
def test_environment_kat(fixture):
    k = np.load(f"{GOLDEN}/{fixture}.npz")
    out = orc.environment(k["rays"], k["scenes"])
    assert np.array_equal(_bits(out), _bits(k["out"]))


@pytest.mark.parametrize("scene", ["ultracomplex", "default", "complex"])
def test_calc_color_kat(scene):
    k = np.load(f"{GOLDEN}/kat_calc_{scene}.npz")
    tris, tonly = load_tris(scene)
    sc, _, _ = setup_from_flags({})
    col, after = orc.calc_color(tris, scene_spheres(scene), sc, tonly, k["rays"], k["seeds"], k["max_bounce"])
    assert np.array_equal(_bits(col), _bits(k["color"]))
    assert np.array_equal(after, k["seed_after"])


@pytest.mark.parametrize("scene", ["ultracomplex", "default"])
def test_calc_debug_color_kat(scene):
    """calcDebugColor (raytracing.c:242-260), the bounce-count integrator (RTC_F_DEBUG_BOUNCES)."""
    k = np.load(f"{GOLDEN}/kat_debug_{scene}.npz")
    tris, tonly = load_tris(scene)
    sc, _, _ = setup_from_flags({})
    col, after = orc.calc_color(tris, scene_spheres(scene), sc, tonly, k["rays"], k["seeds"], k["max_bounce"],
                                debug=True)
    assert np.array_equal(_bits(col), _bits(k["color"]))
    assert np.array_equal(after, k["seed_after"])


GOLD = render_golden()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_render_matches_reference(name, tmp_path):
    """oracle_render == the reference render loop (main.c:81-104) bit for bit: float framebuffer sha256 and
    BMP md5 (BMP written by the product's rtc_write_bmp, pinning it against stbi_write_bmp too)."""
    import raytracingc_amd as rt

    g = GOLD[name]
    tris, tonly = load_tris(g["scene"])
    scene, cam, mb = setup_from_flags(g["flags"])
    d = RtcRenderDesc(g["width"], g["height"], g["spp"], mb, tonly, 0, 1, 0)
    colors, accum, seg = orc.render(tris, scene_spheres(g["scene"]), scene, cam, d, threads=4)
    assert hashlib.sha256(accum.tobytes()).hexdigest() == g["float_sha256"]
    bmp = tmp_path / "o.bmp"
    rt.write_bmp(str(bmp), colors)
    assert hashlib.md5(bmp.read_bytes()).hexdigest() == g["bmp_md5"]


def test_c1_known_answer():
    """simplest 256x256x1 -> BMP md5 3579a190..., float sha256 prefix d2934db26af1ba4d,
    65,944 segments."""
    g = GOLD["C1_simplest_256x256x1"]
    assert g["bmp_md5"] == "3579a1904c5cdf169ddd5ef8c76f1960"
    assert g["float_sha256"].startswith("d2934db26af1ba4d")
    tris, tonly = load_tris("simplest")
    scene, cam, mb = setup_from_flags({})
    _, _, seg = orc.render(tris, None, scene, cam, RtcRenderDesc(256, 256, 1, 10, tonly, 0, 1, 0), threads=4)
    assert seg == 65944


def test_thread_count_and_row_subsets_do_not_change_output():
    tris, tonly = load_tris("fsuzane")
    scene, cam, _ = setup_from_flags({})
    full = RtcRenderDesc(48, 27, 4, 10, tonly, 0, 1, 0)
    _, a1, s1 = orc.render(tris, None, scene, cam, full, threads=1)
    _, a7, s7 = orc.render(tris, None, scene, cam, full, threads=7)
    assert np.array_equal(_bits(a1), _bits(a7)) and s1 == s7
    for start, stride in [(0, 2), (1, 2), (2, 3), (26, 5)]:
        _, part, _ = orc.render(tris, None, scene, cam, RtcRenderDesc(48, 27, 4, 10, tonly, start, stride, 0), threads=3)
        assert np.array_equal(_bits(part), _bits(a1[start::stride]))

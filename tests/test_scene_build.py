"""Host scene build (SURVEY §8 f #1): the product's loaders give the same Triangle[] bytes as the reference's
loaders (loadOBJTriangles raytracing.c:100-147 + objloader.c, parseTriangleFile raytracing.c:76-98), and the
CLI driver keeps main.c's flag / exit-code behaviour."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import REFERENCE, REPO, have_ref_binary, load_tris

import raytracingc_amd as rt

REF_BIN = os.path.join(REPO, "oracle", "_ref", "rtc_ref")
MODELS = os.path.join(REFERENCE, "3Dmodels")
# every model of /root/reference/3Dmodels (objloader.c:340-551 + raytracing.c:100-147)
OBJ_SCENES = ["simplest", "cube", "fsuzane", "complex", "ultracomplex", "rsuzanne", "suze", "4geoms", "simple",
              "withtexture", "suzannes", "asuzane", "plane", "cplane", "fcube", "ccube"]


@pytest.mark.skipif(not os.path.isdir(MODELS), reason="reference models not present (GPU box)")
@pytest.mark.parametrize("name", OBJ_SCENES)
def test_obj_loader_matches_reference(name):
    want, tonly = load_tris(name)
    got = rt.loadOBJTriangles(os.path.join(MODELS, name + ".obj"))
    assert tonly == 1
    assert got.tobytes() == want.tobytes()


def _ref_dump(mode, cwd):
    out = os.path.join(cwd, "dump.tris")
    subprocess.run([REF_BIN, "--dump-tris", mode, out], cwd=cwd, check=True, capture_output=True)
    raw = open(out, "rb").read()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    return np.frombuffer(raw[8:8 + 68 * n], rt.TRIANGLE_DT)


SYNTH_MTL = """# synthetic
newmtl Red
Ns 90.25
Kd 0.9 0.1 0.1
Ke 2.5 0 0
newmtl Glass
Kd 0.2 0.3 1.0
Ns 1000
Ke 0.000000 0.000000 0.000000

newmtl Dim
Kd 0.5 0.5 0.5
Ke 0.25 0.1 0.1
Ns 0
"""

SYNTH_OBJ = """# synthetic quirks: faces before usemtl, unknown material, quads, several normals, blank lines
mtllib synth.mtl
o A
v 1.0 2.0 3.0
v -1.5 0.25 2.0
v 0.5 -0.75 -1.0
v 2.0 2.0 2.0
vn 0.0 1.0 0.0
vn 0.6 0.0 0.8
vt 0 0
f 1/1/1 2/1/2 3/1/1
usemtl Red
f 2/1/2 3/1/1 4/1/2

usemtl Nope
f 1/1/2 2/1/1 3/1/2 4/1/1
usemtl Glass
f 4/1/1 3/1/2 2/1/1
o B
usemtl Dim
v 5 5 5
vn -1 0 0
f 5/1/3 1/1/3 2/1/3
usemtl Red
f 3/1/1 5/1/2 1/1/3
"""


@pytest.mark.skipif(not have_ref_binary(), reason="oracle/_ref/rtc_ref not built")
def test_obj_loader_quirks_match_reference(tmp_path):
    (tmp_path / "synth.mtl").write_text(SYNTH_MTL)
    (tmp_path / "synth.obj").write_text(SYNTH_OBJ)
    want = _ref_dump(str(tmp_path / "synth.obj"), str(tmp_path))
    got = rt.loadOBJTriangles(str(tmp_path / "synth.obj"))
    assert len(got) == 6
    assert got.tobytes() == want.tobytes()


@pytest.mark.skipif(not have_ref_binary(), reason="oracle/_ref/rtc_ref not built")
def test_obj_missing_mtllib_matches_reference(tmp_path):
    (tmp_path / "m.obj").write_text(SYNTH_OBJ.replace("synth.mtl", "absent.mtl"))
    want = _ref_dump(str(tmp_path / "m.obj"), str(tmp_path))
    got = rt.loadOBJTriangles(str(tmp_path / "m.obj"))
    assert got.tobytes() == want.tobytes()
    assert np.all(got["mat"]["color"]["x"] == 1) and np.all(got["mat"]["emissionStrength"] == 0)


TRI_TXT = """Format header with words, digits 3 and symbols: everything but [0-9.+-\\n] is a space
// a comment line 99 99 99
3
{{-5,-5, 5},{-5, 5, 5},{ 5, 5, 5},{{1,1,1},0,0.98}} // trailing comment 7 7
{{ 1.5e0, 2, +3},{-4.25,5,6},{7,8,-9.5},{{0.5,0,1},10,0}}
x/y {{0,0,0},{1,0,0},{0,1,0},{{.1,.2,.3},.5,.75}}
"""


@pytest.mark.skipif(not have_ref_binary(), reason="oracle/_ref/rtc_ref not built")
def test_triangle_file_parser_matches_reference(tmp_path):
    (tmp_path / "triangles.txt").write_text(TRI_TXT)
    want = _ref_dump("default", str(tmp_path))
    got = rt.parseTriangleFile(str(tmp_path / "triangles.txt"))
    assert len(got) == 3
    assert got.tobytes() == want.tobytes()
    assert (tmp_path / "triangles.txt.parsed").exists()


def test_default_triangles_golden_consistent():
    tris, tonly = load_tris("default")
    assert len(tris) == 14 and tonly == 0
    # raytracing.c:24 normals are unit length
    n = np.stack([tris["normal"][c] for c in "xyz"], 1)
    assert np.allclose(np.linalg.norm(n, axis=1), 1, atol=1e-6)


def test_obj_load_failure_is_an_error(tmp_path):
    with pytest.raises(rt.RtcError) as ei:
        rt.loadOBJTriangles(str(tmp_path / "missing.obj"))
    assert ei.value.code == -10003


def test_camera_and_scene_defaults():
    cam = rt.camera_basis()
    ez = np.array([cam.ez.x, cam.ez.y, cam.ez.z])
    ex = np.array([cam.ex.x, cam.ex.y, cam.ex.z])
    assert abs(np.linalg.norm(ez) - 1) < 1e-6 and abs(np.dot(ez, ex)) < 1e-6
    s = rt.default_scene()
    assert s.sunFocus == 22 and abs(s.sunIntensity - 0.75) < 1e-7
    sun = np.array([s.normalizedSunDirection.x, s.normalizedSunDirection.y, s.normalizedSunDirection.z])
    assert np.allclose(sun, np.array([-30, -85, 100]) / np.linalg.norm([-30, -85, 100]), atol=1e-6)


def _cli(args, cwd):
    return subprocess.run([rt.CLI_PATH] + args, cwd=cwd, capture_output=True, text=True)


def test_cli_help_and_errors(tmp_path):
    r = _cli(["-h"], tmp_path)
    assert r.returncode == 0 and "--input" in r.stdout and "--max-bounce" in r.stdout
    r = _cli(["--bogus"], tmp_path)
    assert r.returncode == 0 and 'UNKNOWN ARGUMENT "--bogus"' in r.stderr
    r = _cli(["-s", "10"], tmp_path)
    assert r.returncode == 0 and "--size/-s takes 2 more params" in r.stderr
    r = _cli(["-i", str(tmp_path / "nope.obj")], tmp_path)
    assert r.returncode == 42 and "ERROR WHILE LOADING OBJ" in r.stderr


@pytest.mark.parametrize("name", OBJ_SCENES)
def test_obj_export_round_trip(name, tmp_path):
    """tools/obj_export.write_obj (how bench.py and the CLI tests hand the committed Triangle[] fixtures to the
    reference binary and to the CLI on the GPU box) reproduces the fixture byte for byte through the product's
    loader and, when it is built, through the reference's own loader (rtc_ref --dump-tris)."""
    import sys

    sys.path.insert(0, os.path.join(REPO, "tools"))
    from obj_export import write_obj

    want, _ = load_tris(name)
    obj = str(tmp_path / "scene.obj")
    write_obj(obj, want)
    assert rt.loadOBJTriangles(obj).tobytes() == want.tobytes()
    if have_ref_binary():
        assert _ref_dump(obj, str(tmp_path)).tobytes() == want.tobytes()


def test_bounce_hit_share_probe():
    """rtc_bounce_hit_share (host only): the upload-time probe behind the geometry kernel's workgroups per CU -- a
    scheduling hint, never a change of frame.  Deterministic; the scenes whose bounces hit again (fsuzane) above the
    0.15 threshold, the convex-ish BASELINE scenes well below it; no triangles -> 0; bad arguments refused."""
    import ctypes as C

    shares = {}
    for name in ("fsuzane", "ultracomplex", "complex", "cube"):
        tris, _ = load_tris(name)
        shares[name] = rt.bounce_hit_share(tris)
        assert rt.bounce_hit_share(tris) == shares[name]
    assert shares["fsuzane"] > 0.15
    assert max(shares["ultracomplex"], shares["complex"], shares["cube"]) < 0.05
    assert rt.bounce_hit_share(None) == 0.0
    assert rt.lib().rtc_bounce_hit_share(None, 3, C.byref(C.c_float())) == rt.RTC_EINVAL

#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/ from the reference itself.

Runs oracle/_ref/rtc_ref -- the reference's own C sources (/root/reference) compiled where they lie into
the deterministic variant described in SURVEY.md F4 (oracle/ref_unity.c, oracle/Makefile recipe `make ref`)
-- and records:

  scenes/<name>.tris     Triangle[] produced by the reference loaders (loadOBJTriangles / parseTriangleFile):
                         int32 count, int32 trianglesOnly, count x 68-byte Triangle (raytracing.h:41-45)
  kat_rng.npz            RandomValue / RandomValueNormalDistrubtion / RandomDiretion sequences per seed
  kat_tri.npz            rayTriangle on random + constructed edge-case (ray, triangle) pairs
  kat_sphere.npz         raySphere
  kat_env.npz            getEnvironmentLight
  kat_env_edge.npz       getEnvironmentLight at signed zeros, special sun intensities / focus values
  kat_calc_<scene>.npz   calcColor per (ray, seed, maxBounce)
  kat_debug_<scene>.npz  calcDebugColor (raytracing.c:242-260) per (ray, seed, maxBounce)
  render_golden.json     full renders (main.c render loop): sha256 of the pre-quantisation float
                         framebuffer and md5 of the BMP, per configuration

Only this script reads /root/reference (model files as inputs); it runs in the build container, never on
the GPU box.  Re-run with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from raytracingc_amd._abi import RAY_DT, SCENE_DT, SPHERE_DT, TRIANGLE_DT  # noqa: E402

REF_DIR = os.environ.get("RTC_REFERENCE", "/root/reference")
MODELS = os.path.join(REF_DIR, "3Dmodels")
REF_BIN = os.path.join(REPO, "oracle", "_ref", "rtc_ref")

# scenes used by the BASELINE configs plus loader-quirk scenes (quads: suze; missing mtllib: simple;
# several materials: rsuzanne, withtexture; mixed: 4geoms)
OBJ_SCENES = ["simplest", "cube", "fsuzane", "complex", "ultracomplex", "rsuzanne", "suze", "4geoms", "simple",
              "withtexture", "suzannes", "asuzane", "plane", "cplane", "fcube", "ccube"]

KAT_KEYS = {}


def run_ref(args, cwd):
    r = subprocess.run([REF_BIN] + args, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if r.returncode != 0:
        raise RuntimeError(f"rtc_ref {' '.join(args)} failed: {r.stderr.decode()[-500:]}")
    return r


def mode_arg(scene: str) -> str:
    return "default" if scene == "default" else os.path.join(MODELS, scene + ".obj")


def gen_scenes(work):
    os.makedirs(os.path.join(HERE, "scenes"), exist_ok=True)
    for s in OBJ_SCENES + ["default"]:
        out = os.path.join(HERE, "scenes", s + ".tris")
        run_ref(["--dump-tris", mode_arg(s), out], work)


def rand_unit(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def gen_kat_rng(work):
    seeds = np.array([0, 1, 2, 7, 12345, 65535, 2**31 - 1, 2**31, 2**32 - 1, 1920 * 1080 - 1, 3840 * 2160 - 1,
                      0xDEADBEEF], np.uint32)
    draws = 96
    uni, nrm, dirs = [], [], []
    for s in seeds:
        out = os.path.join(work, "rng.bin")
        run_ref(["--kat-rng", str(int(s)), str(draws), out], work)
        a = np.fromfile(out, np.float32)
        uni.append(a[:draws])
        nrm.append(a[draws:2 * draws])
        dirs.append(a[2 * draws:].reshape(draws, 3))
    np.savez_compressed(os.path.join(HERE, "kat_rng.npz"), seeds=seeds, uniform=np.array(uni), normal=np.array(nrm),
                        direction=np.array(dirs))


def gen_kat_tri(work, rng):
    n_rand = 3000
    rays = np.zeros(n_rand, RAY_DT)
    tris = np.zeros(n_rand, TRIANGLE_DT)
    P = rng.uniform(-3, 3, size=(n_rand, 3)).astype(np.float32)
    A = rng.uniform(-2, 2, size=(n_rand, 3)).astype(np.float32)
    B = (A + rng.uniform(-2, 2, size=(n_rand, 3))).astype(np.float32)
    Cc = (A + rng.uniform(-2, 2, size=(n_rand, 3))).astype(np.float32)
    # aim a fraction of rays at a point inside the triangle so hits occur
    bary = rng.dirichlet([1, 1, 1], size=n_rand).astype(np.float32)
    target = bary[:, :1] * A + bary[:, 1:2] * B + bary[:, 2:] * Cc
    d = target - P
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    aim = rng.random(n_rand) < 0.6
    dirs = np.where(aim[:, None], d, rand_unit(rng, n_rand)).astype(np.float32)
    nrm = np.cross(B - A, Cc - A)
    nrm = nrm / np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
    flip = rng.random(n_rand) < 0.5
    nrm = np.where(flip[:, None], -nrm, nrm).astype(np.float32)
    for f, arr in (("x", 0), ("y", 1), ("z", 2)):
        rays["pos"][f], rays["dir"][f] = P[:, arr], dirs[:, arr]
        tris["posA"][f], tris["posB"][f], tris["posC"][f] = A[:, arr], B[:, arr], Cc[:, arr]
        tris["normal"][f] = nrm[:, arr]
    # constructed edge cases on the unit triangle A=(0,0,0) B=(1,0,0) C=(0,1,0), normal (0,0,-1), ray along +z
    edge = []

    def add(pos, dir_, a=(0, 0, 0), b=(1, 0, 0), c=(0, 1, 0), n=(0, 0, -1)):
        edge.append((pos, dir_, a, b, c, n))

    z0 = -1.0
    for (x, y) in [(0, 0), (1, 0), (0, 1), (0.5, 0.5), (0.25, 0.75), (1e-8, 0), (0, 1e-8), (-1e-8, 0.5), (0.5, -1e-8),
                   (0.5000001, 0.5), (0.3, 0.7), (0.7, 0.3000001), (0.999999, 1e-6)]:
        add((x, y, z0), (0, 0, 1))
    for dz in [0.001, 0.0009999999, 0.0010000001, 0.00099999, 0.0011, 0.0, -0.001, 1e-30]:
        add((0.2, 0.2, -dz), (0, 0, 1))  # dst ~= EPSILON
    for t in [1e-3, 9.99e-4, 1.001e-3, 5e-4, 2e-3]:
        # det = dot(AB, dir x AC) = dir.z for this triangle: grazing directions around |det| = EPSILON
        dvec = np.array([np.sqrt(max(0.0, 1 - t * t)), 0.0, t])
        add((0.2 - dvec[0] * 10, 0.2, -dvec[2] * 10), tuple(dvec))
    add((0.2, 0.2, -1), (0, 0, -1))  # back face: dot(dir, N) > 0
    add((0.2, 0.2, -1), (1, 0, 0))  # dot == 0 exactly -> culled
    add((0.2, 0.2, -1), (float("nan"), 0, 1))
    add((0.2, 0.2, -1), (0, 0, float("inf")))
    add((0.2, 0.2, -1), (0, 0, 1), a=(0, 0, 0), b=(1, 1, 0), c=(2, 2, 0))  # degenerate
    add((0.2, 0.2, -1e6), (0, 0, 1))
    add((1e7, 1e7, -1), (0, 0, 1), a=(1e7, 1e7, 0), b=(1e7 + 1, 1e7, 0), c=(1e7, 1e7 + 1, 0))
    erays = np.zeros(len(edge), RAY_DT)
    etris = np.zeros(len(edge), TRIANGLE_DT)
    for i, (p, dd, a, b, c, n) in enumerate(edge):
        for k, f in enumerate("xyz"):
            erays["pos"][f][i], erays["dir"][f][i] = p[k], dd[k]
            etris["posA"][f][i], etris["posB"][f][i], etris["posC"][f][i] = a[k], b[k], c[k]
            etris["normal"][f][i] = n[k]
    rays = np.concatenate([rays, erays])
    tris = np.concatenate([tris, etris])
    kin = np.zeros(len(rays), np.dtype([("ray", RAY_DT), ("t", TRIANGLE_DT)]))
    kin["ray"], kin["t"] = rays, tris
    fi, fo = os.path.join(work, "tri.in"), os.path.join(work, "tri.out")
    kin.tofile(fi)
    run_ref(["--kat-tri", fi, fo], work)
    out = np.fromfile(fo, np.dtype([("didHit", "<i4"), ("dst", "<f4"), ("normal", "<f4", 3)]))
    np.savez_compressed(os.path.join(HERE, "kat_tri.npz"), rays=rays, tris=tris, didHit=out["didHit"],
                        dst=out["dst"])


def gen_kat_sphere(work, rng):
    n = 2000
    rays = np.zeros(n, RAY_DT)
    sph = np.zeros(n, SPHERE_DT)
    P = rng.uniform(-6, 6, size=(n, 3)).astype(np.float32)
    Cc = rng.uniform(-2, 2, size=(n, 3)).astype(np.float32)
    R = rng.uniform(0.1, 3, size=n).astype(np.float32)
    d = Cc - P + rng.normal(scale=1.0, size=(n, 3)).astype(np.float32)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    inside = rng.random(n) < 0.15
    P = np.where(inside[:, None], Cc, P)  # origins at the centre -> far root
    for k, f in enumerate("xyz"):
        rays["pos"][f], rays["dir"][f] = P[:, k], d[:, k]
        sph["pos"][f] = Cc[:, k]
    sph["r"] = R
    # the default scene's sphere (scene.h:17-19) from the default camera, and tangent / surface cases
    extra = [((-4.75, -1.5, -4.75), (0.6, 0.1, 0.8), (0, 1, 0), 2.5), ((0, 1, -2.5), (0, 0, 1), (0, 1, 0), 2.5),
             ((0, 1 + 2.5, -10), (0, 0, 1), (0, 1, 0), 2.5), ((0, 1, 2.5 + 0.0005), (0, 0, -1), (0, 1, 0), 2.5),
             ((0, 1, 2.5 - 0.0005), (0, 0, 1), (0, 1, 0), 2.5)]
    er = np.zeros(len(extra), RAY_DT)
    es = np.zeros(len(extra), SPHERE_DT)
    for i, (p, dd, c, r) in enumerate(extra):
        dd = np.array(dd, np.float64)
        dd = dd / np.linalg.norm(dd)
        for k, f in enumerate("xyz"):
            er["pos"][f][i], er["dir"][f][i], es["pos"][f][i] = p[k], dd[k], c[k]
        es["r"][i] = r
    rays = np.concatenate([rays, er])
    sph = np.concatenate([sph, es])
    kin = np.zeros(len(rays), np.dtype([("ray", RAY_DT), ("c", "<f4", 3), ("r", "<f4")]))
    kin["ray"] = rays
    kin["c"] = np.stack([sph["pos"]["x"], sph["pos"]["y"], sph["pos"]["z"]], 1)
    kin["r"] = sph["r"]
    fi, fo = os.path.join(work, "sph.in"), os.path.join(work, "sph.out")
    kin.tofile(fi)
    run_ref(["--kat-sphere", fi, fo], work)
    out = np.fromfile(fo, np.dtype([("didHit", "<i4"), ("dst", "<f4"), ("hitPoint", "<f4", 3), ("normal", "<f4", 3)]))
    np.savez_compressed(os.path.join(HERE, "kat_sphere.npz"), rays=rays, spheres=sph, didHit=out["didHit"],
                        dst=out["dst"], normal=out["normal"])


def gen_kat_env(work, rng):
    n = 4000
    rays = np.zeros(n, RAY_DT)
    d = rand_unit(rng, n)
    # concentrate some directions near the horizon and near the sun
    d[:400, 1] = rng.uniform(-0.02, 0.02, 400).astype(np.float32)
    sun = np.array([-30, -85, 100], np.float64)
    sun = (sun / np.linalg.norm(sun)).astype(np.float32)
    jit = (sun[None, :] + rng.normal(scale=0.05, size=(400, 3))).astype(np.float32)
    d[400:800] = jit / np.linalg.norm(jit, axis=1, keepdims=True)
    d[800] = (0, 0, 1)
    d[801] = (0, -0.0, 1)
    d[802] = (0, 1, 0)
    d[803] = (0, -1, 0)
    d[804] = (np.nan, np.nan, np.nan)
    for k, f in enumerate("xyz"):
        rays["dir"][f] = d[:, k]
    scenes = np.zeros(n, SCENE_DT)

    def setv(name, rows, v):
        for k, f in enumerate("xyz"):
            scenes[name][f][rows] = v[:, k] if np.ndim(v) == 2 else v[k]

    setv("normalizedSunDirection", slice(None), sun)
    setv("skyColorHorizon", slice(None), np.array([1, 1, 1], np.float32))
    setv("skyColorZenith", slice(None), np.array([0.263, 0.969, 0.871], np.float32))
    setv("groundColor", slice(None), np.array([0.66, 0.66, 0.66], np.float32))
    scenes["sunFocus"] = 22
    scenes["sunIntensity"] = np.float32(0.75)
    # a quarter of the records use random sky / sun parameters (the CLI's -gc/-sch/-scz/--sun)
    m = slice(3000, 4000)
    s2 = rand_unit(rng, 1000)
    setv("normalizedSunDirection", m, s2)
    setv("skyColorHorizon", m, rng.random((1000, 3)).astype(np.float32))
    setv("skyColorZenith", m, rng.random((1000, 3)).astype(np.float32))
    setv("groundColor", m, rng.random((1000, 3)).astype(np.float32))
    scenes["sunFocus"][m] = rng.choice(np.array([0, 1, 3, 7.5, 22, 100], np.float32), 1000)
    scenes["sunIntensity"][m] = rng.uniform(0, 3, 1000).astype(np.float32)
    kin = np.zeros(n, np.dtype([("ray", RAY_DT), ("s", SCENE_DT)]))
    kin["ray"], kin["s"] = rays, scenes
    fi, fo = os.path.join(work, "env.in"), os.path.join(work, "env.out")
    kin.tofile(fi)
    run_ref(["--kat-env", fi, fo], work)
    out = np.fromfile(fo, np.float32).reshape(n, 3)
    np.savez_compressed(os.path.join(HERE, "kat_env.npz"), rays=rays, scenes=scenes, out=out)


def camera_rays(w, h, pixels):
    """Primary rays of the default camera (main.c:88-94, 114-116, 252-255) in float32, x,y pixel pairs."""
    from raytracingc_amd import camera_basis  # the product's host camera (pinned by render hashes)

    cam = camera_basis()
    ex = np.array([cam.ex.x, cam.ex.y, cam.ex.z], np.float32)
    ey = np.array([cam.ey.x, cam.ey.y, cam.ey.z], np.float32)
    ez = np.array([cam.ez.x, cam.ez.y, cam.ez.z], np.float32)
    rays = np.zeros(len(pixels), RAY_DT)
    for i, (x, y) in enumerate(pixels):
        dx = np.float32(x - w // 2) / np.float32(h // 2)
        dy = np.float32(y - h // 2) / np.float32(h // 2)
        d = (ex * dx + ey * dy) + ez * np.float32(cam.fov)
        inv = np.float32(1.0 / float(np.float32(np.sqrt(np.float64(np.float32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))))
        d = d * inv
        rays["pos"]["x"][i], rays["pos"]["y"][i], rays["pos"]["z"][i] = cam.origin.x, cam.origin.y, cam.origin.z
        rays["dir"]["x"][i], rays["dir"]["y"][i], rays["dir"]["z"][i] = d
    return rays


def gen_kat_calc(work, rng, scene, debug=False):
    w, h = 480, 270
    # pixels where geometry is visible (rows 26-192 hold hits for the OBJ scenes)
    pix = [(int(x), int(y)) for x, y in zip(rng.integers(0, w, 600), rng.integers(20, 200, 600))]
    rays = camera_rays(w, h, pix)
    # plus random rays from inside the scene volume
    n2 = 200
    rr = np.zeros(n2, RAY_DT)
    pos = rng.uniform(-2, 2, size=(n2, 3)).astype(np.float32)
    d = rand_unit(rng, n2)
    for k, f in enumerate("xyz"):
        rr["pos"][f], rr["dir"][f] = pos[:, k], d[:, k]
    rays = np.concatenate([rays, rr])
    n = len(rays)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    mb = rng.choice(np.array([0, 1, 2, 3, 10, 10, 10, 25], np.int32), n)
    kin = np.zeros(n, np.dtype([("ray", RAY_DT), ("seed", "<u4"), ("mb", "<i4")]))
    kin["ray"], kin["seed"], kin["mb"] = rays, seeds, mb
    fi, fo = os.path.join(work, "calc.in"), os.path.join(work, "calc.out")
    kin.tofile(fi)
    run_ref(["--kat-debug" if debug else "--kat-calc", mode_arg(scene), fi, fo], work)
    out = np.fromfile(fo, np.dtype([("color", "<f4", 3), ("seedAfter", "<u4")]))
    np.savez_compressed(os.path.join(HERE, f"kat_{'debug' if debug else 'calc'}_{scene}.npz"), rays=rays, seeds=seeds,
                        max_bounce=mb, color=out["color"], seed_after=out["seedAfter"])


# (name, scene, W, H, spp, extra reference flags)
RENDER_CONFIGS = [("C1_simplest_256x256x1", "simplest", 256, 256, 1, [])]
for _s in ["cube", "fsuzane", "complex", "ultracomplex", "default", "rsuzanne"]:
    for _spp in (1, 4, 16):
        RENDER_CONFIGS.append((f"{_s}_64x36x{_spp}", _s, 64, 36, _spp, []))
    RENDER_CONFIGS.append((f"{_s}_160x90x4", _s, 160, 90, 4, []))
RENDER_CONFIGS += [
    ("ultracomplex_cam_96x64x8", "ultracomplex", 96, 64, 8, ["-p", "3", "-2", "-5", "-t", "0", "-1", "0", "-f", "1.3",
                                                             "-b", "4"]),
    ("default_sky_80x60x8", "default", 80, 60, 8, ["--sun", "10", "-50", "30", "8", "1.2", "-gc", ".2", ".3", ".4",
                                                   "-sch", ".9", ".8", ".7", "-scz", ".1", ".2", ".9"]),
    ("fsuzane_odd_33x17x3", "fsuzane", 33, 17, 3, []),
    ("complex_1x1x5", "complex", 1, 1, 5, []),
    ("cube_7x1x2", "cube", 7, 1, 2, []),
    ("default_b0_32x18x4", "default", 32, 18, 4, ["-b", "0"]),
    ("default_b1_32x18x4", "default", 32, 18, 4, ["-b", "1"]),
    ("ultracomplex_spp0_16x9x0", "ultracomplex", 16, 9, 0, []),
    ("suze_quads_64x36x4", "suze", 64, 36, 4, []),
    ("4geoms_64x36x4", "4geoms", 64, 36, 4, []),
    ("withtexture_64x36x4", "withtexture", 64, 36, 4, []),
    # the remaining reference models: suzannes.obj (5,208 triangles, the largest, > 256 = the general kernel),
    # asuzane, plane, cplane, fcube, ccube
    ("suzannes_96x54x4", "suzannes", 96, 54, 4, []),
    ("suzannes_cam_64x48x2", "suzannes", 64, 48, 2, ["-p", "-3", "-1", "-3", "-t", "0", "-0.5", "0", "-b", "3"]),
    ("asuzane_64x36x4", "asuzane", 64, 36, 4, []),
    ("plane_64x36x4", "plane", 64, 36, 4, []),
    ("cplane_64x36x4", "cplane", 64, 36, 4, []),
    ("fcube_64x36x4", "fcube", 64, 36, 4, []),
    ("ccube_64x36x4", "ccube", 64, 36, 4, []),
]


def parse_flags(extra):
    """The reference CLI flags used above -> a dict the tests turn into Scene/RtcCamera/maxBounce."""
    cfg = {}
    i = 0
    while i < len(extra):
        f = extra[i]
        if f == "-p":
            cfg["origin"] = [float(v) for v in extra[i + 1:i + 4]]
            i += 4
        elif f == "-t":
            cfg["looking_at"] = [float(v) for v in extra[i + 1:i + 4]]
            i += 4
        elif f == "-f":
            cfg["fov"] = float(extra[i + 1])
            i += 2
        elif f == "-b":
            cfg["max_bounce"] = int(extra[i + 1])
            i += 2
        elif f == "--sun":
            cfg["sun"] = [float(v) for v in extra[i + 1:i + 4]]
            cfg["focus"], cfg["intensity"] = float(extra[i + 4]), float(extra[i + 5])
            i += 6
        elif f in ("-gc", "-sch", "-scz"):
            cfg[{"-gc": "ground", "-sch": "horizon", "-scz": "zenith"}[f]] = [float(v) for v in extra[i + 1:i + 4]]
            i += 4
        else:
            raise ValueError(f)
    return cfg


def gen_renders(work):
    out = {}
    for name, scene, w, h, spp, extra in RENDER_CONFIGS:
        fb = os.path.join(work, "fb.f32")
        bmp = os.path.join(work, "out.bmp")
        if os.path.exists(fb):
            os.remove(fb)
        run_ref(["--spp", str(spp), "--dump-float", fb, "-i", mode_arg(scene), "-s", str(w), str(h), "-o", bmp]
                + extra if scene != "default" else
                ["--spp", str(spp), "--dump-float", fb, "-s", str(w), str(h), "-o", bmp] + extra, work)
        raw = open(fb, "rb").read() if os.path.exists(fb) else b""
        data = raw[8:]
        out[name] = {
            "scene": scene, "width": w, "height": h, "spp": spp, "flags": parse_flags(extra),
            "float_sha256": hashlib.sha256(data).hexdigest(),
            "bmp_md5": hashlib.md5(open(bmp, "rb").read()).hexdigest(),
        }
        print(f"{name}: {out[name]['bmp_md5']}")
    with open(os.path.join(HERE, "render_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def gen_meta():
    """Where the fixtures came from: the glibc whose libm the reference called (powf/log/cos) and the CPU
    features that decide glibc's ifunc choice (x86-64 powf/log/cos pick their FMA builds when the CPU has
    FMA + AVX2; rtc_math.h restates the FMA build of powf)."""
    import platform

    flags = set()
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags") and not flags:
                flags = set(line.split(":", 1)[1].split())
            if line.startswith("model name") and not model:
                model = line.split(":", 1)[1].strip()
    except OSError:
        pass
    meta = {
        "glibc": platform.libc_ver()[1],
        "cpu_model": model,
        "cpu_fma": "fma" in flags,
        "cpu_avx2": "avx2" in flags,
        "libm_ifunc": "FMA builds of powf/log/cos (fma+avx2 present)" if {"fma", "avx2"} <= flags
                      else "generic SSE2 builds (no fma/avx2): the device powf restates the FMA build",
        "compiler": subprocess.run(["gcc", "--version"], capture_output=True, text=True).stdout.splitlines()[0],
        "ref_binary": "oracle/_ref/rtc_ref (make ref: gcc -O3 on /root/reference sources via oracle/ref_unity.c)",
    }
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def gen_kat_env_edge(work):
    """getEnvironmentLight at the values where a powf's result is known without evaluating it (the device
    skips those powf calls wave by wave): rays below the horizon, the sun behind the ray, signed zeros, a
    negative / zero / infinite / NaN sun intensity, sun focus 0, odd integers, fractions and negatives."""
    rng = np.random.default_rng(20261016)
    n = 4096
    d = rand_unit(rng, n)
    d[:512, 1] = np.abs(d[:512, 1])  # below the horizon (+y is down after the loader's flip)
    d[512:1024, 1] = -np.abs(d[512:1024, 1])
    zeros = np.array([[0, 0, 0], [-0.0, -0.0, -0.0], [0, -0.0, 0], [-0.0, 0, -0.0], [0, 0, 1], [0, -0.0, 1],
                      [0, 0, -1], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, -0.0, -1]], np.float32)
    d[1024:1024 + len(zeros)] = zeros
    d[1100:1200] = np.nan
    rays = np.zeros(n, RAY_DT)
    for k, f in enumerate("xyz"):
        rays["dir"][f] = d[:, k]
    scenes = np.zeros(n, SCENE_DT)

    def setv(name, v):
        for k, f in enumerate("xyz"):
            scenes[name][f] = v[:, k]

    sun = rand_unit(rng, n)
    sun[::7] = d[::7]  # the sun along the ray, and opposite it
    sun[3::7] = -d[3::7]
    sun[5::11] = np.array([0, 0, 0], np.float32)
    sun = np.where(np.isnan(sun), np.float32(0), sun)
    setv("normalizedSunDirection", sun)
    setv("skyColorHorizon", rng.random((n, 3)).astype(np.float32))
    setv("skyColorZenith", rng.random((n, 3)).astype(np.float32))
    g = rng.random((n, 3)).astype(np.float32)
    g[::13] = np.float32(-0.0)
    g[1::13] = np.float32(0.0)
    setv("groundColor", g)
    scenes["sunFocus"] = rng.choice(np.array([0, 1, 2, 3, 5, 7.5, 22, 100, -1, -3, 0.5, 1e-30], np.float32), n)
    scenes["sunIntensity"] = rng.choice(np.array([0.75, -0.75, 0, -0.0, np.inf, -np.inf, np.nan, 3, 1e30],
                                                 np.float32), n)
    kin = np.zeros(n, np.dtype([("ray", RAY_DT), ("s", SCENE_DT)]))
    kin["ray"], kin["s"] = rays, scenes
    fi, fo = os.path.join(work, "env_edge.in"), os.path.join(work, "env_edge.out")
    kin.tofile(fi)
    run_ref(["--kat-env", fi, fo], work)
    out = np.fromfile(fo, np.float32).reshape(n, 3)
    np.savez_compressed(os.path.join(HERE, "kat_env_edge.npz"), rays=rays, scenes=scenes, out=out)


def main():
    if not os.path.exists(REF_BIN):
        sys.exit(f"{REF_BIN} missing: run `make ref` (needs {REF_DIR})")
    if sys.argv[1:] == ["--env-edge"]:  # the one fixture added later (its own seed; the others unchanged)
        with tempfile.TemporaryDirectory() as work:
            gen_kat_env_edge(work)
        return
    rng = np.random.default_rng(20251003)
    with tempfile.TemporaryDirectory() as work:
        # default mode reads ./triangles.txt (main.c:237): give the reference a private working dir
        shutil.copy(os.path.join(REF_DIR, "triangles.txt"), os.path.join(work, "triangles.txt"))
        gen_scenes(work)
        gen_kat_rng(work)
        gen_kat_tri(work, rng)
        gen_kat_sphere(work, rng)
        gen_kat_env(work, rng)
        for s in ["ultracomplex", "default", "complex"]:
            gen_kat_calc(work, rng, s)
        for s in ["ultracomplex", "default"]:
            gen_kat_calc(work, rng, s, debug=True)
        gen_renders(work)
        gen_kat_env_edge(work)
        gen_meta()


if __name__ == "__main__":
    main()

"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference render path (oracle/rtc_oracle.c).  Only tests/, the smoke() check of
__graft_entry__ and bench.py's cpu_baseline leg may use it, and only as the checker / the timed CPU
baseline.  The product (raytracingc_amd, librtc.so) never loads it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from raytracingc_amd._abi import (RAY_DT, SCENE_DT, SPHERE_DT, TRIANGLE_DT, RtcCamera, RtcRenderDesc, Scene)

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(HERE, "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "rtc_ref")

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError(f"{ORACLE_LIB} not built; run `make`")
        L = C.CDLL(ORACLE_LIB)
        vp, ip, sz = C.c_void_p, C.c_int, C.c_size_t
        L.oracle_render.argtypes = [vp, ip, vp, ip, C.POINTER(Scene), C.POINTER(RtcCamera), C.POINTER(RtcRenderDesc),
                                    ip, vp, vp, C.POINTER(C.c_ulonglong)]
        L.oracle_rows_selected.argtypes = [C.POINTER(RtcRenderDesc)]
        L.oracle_ray_triangle.argtypes = [vp, vp, sz, vp, vp]
        L.oracle_ray_triangle.restype = None
        L.oracle_ray_sphere.argtypes = [vp, vp, sz, vp, vp, vp]
        L.oracle_ray_sphere.restype = None
        L.oracle_environment.argtypes = [vp, vp, sz, vp]
        L.oracle_environment.restype = None
        L.oracle_random.argtypes = [vp, sz, ip, vp, vp, vp]
        L.oracle_random.restype = None
        L.oracle_calc_color.argtypes = [vp, ip, vp, ip, C.POINTER(Scene), ip, vp, vp, vp, sz, vp, vp, ip]
        L.oracle_calc_color.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _arr(a, dt):
    if a is None or len(a) == 0:
        return None, 0
    a = np.ascontiguousarray(a, dtype=dt)
    return a, len(a)


def render(tris, spheres, scene: Scene, cam: RtcCamera, desc: RtcRenderDesc, threads: int = 8):
    """oracle_render: the reference render loop on CPU threads (row-interleaved like main.c:84).
    Returns (colors uint8 [rows, W, 3], accum float32 [rows, W, 3], segments)."""
    t, nt = _arr(tris, TRIANGLE_DT)
    s, ns = _arr(spheres, SPHERE_DT)
    rows = lib().oracle_rows_selected(C.byref(desc))
    colors = np.zeros((rows, desc.width, 3), np.uint8)
    accum = np.zeros((rows, desc.width, 3), np.float32)
    seg = C.c_ulonglong(0)
    rc = lib().oracle_render(_p(t), nt, _p(s), ns, C.byref(scene), C.byref(cam), C.byref(desc), threads, _p(colors),
                             _p(accum), C.byref(seg))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed ({rc})")
    return colors, accum, seg.value


def ray_triangle(rays, tris):
    r = np.ascontiguousarray(rays, RAY_DT)
    t = np.ascontiguousarray(tris, TRIANGLE_DT)
    n = len(r)
    hit, dst = np.zeros(n, np.int32), np.zeros(n, np.float32)
    lib().oracle_ray_triangle(_p(r), _p(t), n, _p(hit), _p(dst))
    return hit, dst


def ray_sphere(rays, spheres):
    r = np.ascontiguousarray(rays, RAY_DT)
    s = np.ascontiguousarray(spheres, SPHERE_DT)
    n = len(r)
    hit, dst, nrm = np.zeros(n, np.int32), np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    lib().oracle_ray_sphere(_p(r), _p(s), n, _p(hit), _p(dst), _p(nrm))
    return hit, dst, nrm


def environment(rays, scenes):
    r = np.ascontiguousarray(rays, RAY_DT)
    s = np.ascontiguousarray(scenes, SCENE_DT)
    n = len(r)
    out = np.zeros((n, 3), np.float32)
    lib().oracle_environment(_p(r), _p(s), n, _p(out))
    return out


def random_sequences(seeds, draws: int):
    sd = np.ascontiguousarray(seeds, np.uint32)
    n = len(sd)
    u = np.zeros((n, draws), np.float32)
    g = np.zeros((n, draws), np.float32)
    d = np.zeros((n, draws, 3), np.float32)
    lib().oracle_random(_p(sd), n, draws, _p(u), _p(g), _p(d))
    return u, g, d


def calc_color(tris, spheres, scene: Scene, triangles_only: int, rays, seeds, max_bounce, debug: bool = False):
    t, nt = _arr(tris, TRIANGLE_DT)
    s, ns = _arr(spheres, SPHERE_DT)
    r = np.ascontiguousarray(rays, RAY_DT)
    sd = np.ascontiguousarray(seeds, np.uint32)
    mb = np.ascontiguousarray(max_bounce, np.int32)
    n = len(r)
    out = np.zeros((n, 3), np.float32)
    after = np.zeros(n, np.uint32)
    lib().oracle_calc_color(_p(t), nt, _p(s), ns, C.byref(scene), triangles_only, _p(r), _p(sd), _p(mb), n, _p(out),
                            _p(after), int(debug))
    return out, after

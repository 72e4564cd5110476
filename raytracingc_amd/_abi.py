"""ctypes mirror of include/rtc.h (the C ABI of librtc.so).

Struct layouts are the reference's (raytracing.h:7-69, moremath.h:10-13); the numpy dtypes below have
the same byte layout so Triangle[] / Sphere[] arrays cross the boundary without conversion.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RTC_LIB_PATH selects another build of the library (e.g. the diagnostic librtc_diag.so for tools/chain_sections.py)
LIB_PATH = os.environ.get("RTC_LIB_PATH") or os.path.join(HERE, "_lib", "librtc.so")
CLI_PATH = os.path.join(HERE, "_lib", "rtc")


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Scene(C.Structure):  # raytracing.h:7-11
    _fields_ = [
        ("normalizedSunDirection", Vec3),
        ("skyColorHorizon", Vec3),
        ("skyColorZenith", Vec3),
        ("groundColor", Vec3),
        ("sunFocus", C.c_float),
        ("sunIntensity", C.c_float),
    ]


class Material(C.Structure):  # raytracing.h:25-30
    _fields_ = [("color", Vec3), ("emissionStrength", C.c_float), ("smoothness", C.c_float)]


class Sphere(C.Structure):  # raytracing.h:34-39
    _fields_ = [("pos", Vec3), ("r", C.c_float), ("mat", Material)]


class Triangle(C.Structure):  # raytracing.h:41-45
    _fields_ = [("posA", Vec3), ("posB", Vec3), ("posC", Vec3), ("normal", Vec3), ("mat", Material)]


class Ray(C.Structure):  # raytracing.h:64-68
    _fields_ = [("pos", Vec3), ("dir", Vec3)]


class RtcCamera(C.Structure):
    _fields_ = [("origin", Vec3), ("ex", Vec3), ("ey", Vec3), ("ez", Vec3), ("fov", C.c_float)]


class RtcRenderDesc(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("spp", C.c_int),
        ("maxBounce", C.c_int),
        ("trianglesOnly", C.c_int),
        ("rowStart", C.c_int),
        ("rowStride", C.c_int),
        ("flags", C.c_int),
        ("rowBand", C.c_int),  # rows per interleaved band (rtc.h; 0 or 1: single rows)
    ]


class RtcStats(C.Structure):
    _fields_ = [
        ("renderMs", C.c_double),
        ("totalMs", C.c_double),
        ("segments", C.c_ulonglong),
        ("samples", C.c_ulonglong),
        ("triTests", C.c_ulonglong),
        ("clusterTests", C.c_ulonglong),
        ("discardedTests", C.c_ulonglong),
        ("frameMs", C.c_double),
    ]


class RtcLoopStats(C.Structure):
    _fields_ = [
        ("wallMs", C.c_double),
        ("frames", C.c_int),
        ("enqueueMs", C.c_double),
        ("copyMsMedian", C.c_double),
        ("copyMsMax", C.c_double),
    ]


RTC_F_HOIST_PRIMARY = 0x1
RTC_F_DEBUG_BOUNCES = 0x2
RTC_F_NO_TILE_CULL = 0x4
RTC_F_NO_REORDER = 0x8
RTC_F_NO_COOP = 0x10
RTC_F_NO_CLUSTER_CULL = 0x20
RTC_F_COOP4 = 0x40  # removed kernels: RTC_EINVAL
RTC_F_COOP8 = 0x80
RTC_F_SPEC = 0x100
RTC_F_PIPE = 0x200
RTC_F_CHAIN_INLINE = 0x400
RTC_F_OVERLAP = 0x800
RTC_F_HOST_ROWS = 0x1000
RTC_SEGMENT_COUNTERS = 5  # u64 counters rtc_render_rows_async adds to (include/rtc.h)
RTC_EINVAL, RTC_ENODEV, RTC_EIO, RTC_ENOMEM, RTC_EFORMAT = -10001, -10002, -10003, -10004, -10005
RTC_ETIMEDOUT, RTC_EBUSY = -10006, -10007

assert C.sizeof(Vec3) == 12 and C.sizeof(Scene) == 56 and C.sizeof(Material) == 20
assert C.sizeof(Sphere) == 36 and C.sizeof(Triangle) == 68 and C.sizeof(Ray) == 24

# numpy views with identical byte layouts
VEC3_DT = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4")])
MATERIAL_DT = np.dtype([("color", VEC3_DT), ("emissionStrength", "<f4"), ("smoothness", "<f4")])
TRIANGLE_DT = np.dtype(
    [("posA", VEC3_DT), ("posB", VEC3_DT), ("posC", VEC3_DT), ("normal", VEC3_DT), ("mat", MATERIAL_DT)]
)
SPHERE_DT = np.dtype([("pos", VEC3_DT), ("r", "<f4"), ("mat", MATERIAL_DT)])
RAY_DT = np.dtype([("pos", VEC3_DT), ("dir", VEC3_DT)])
SCENE_DT = np.dtype(
    [
        ("normalizedSunDirection", VEC3_DT),
        ("skyColorHorizon", VEC3_DT),
        ("skyColorZenith", VEC3_DT),
        ("groundColor", VEC3_DT),
        ("sunFocus", "<f4"),
        ("sunIntensity", "<f4"),
    ]
)
assert TRIANGLE_DT.itemsize == 68 and SPHERE_DT.itemsize == 36 and RAY_DT.itemsize == 24
assert SCENE_DT.itemsize == 56

# every symbol include/rtc.h declares (tests check the library exports all of them)
EXPORTS = [
    "rtc_last_error", "rtc_version", "rtc_device_count",
    "rtc_load_obj", "rtc_parse_triangle_file", "rtc_free", "rtc_default_spheres", "rtc_default_scene",
    "rtc_scene_set_sun", "rtc_camera_basis", "rtc_write_bmp", "rtc_quantize",
    "rtc_render", "rtc_render_multi", "rtc_last_multi_info",
    "rtc_scene_upload", "rtc_scene_release", "rtc_rows_selected", "rtc_render_rows_async", "rtc_scene_set_timing", "rtc_scene_kernel_times",
    "rtc_bounce_hit_share", "rtc_scene_chain_wgs",
    "rtc_scene_set_geometry_event", "rtc_scene_set_frame_event",
    "rtc_deinterleave_async", "rtc_deinterleave_bands_async", "rtc_copy_async", "rtc_copy_d2h_dma", "rtc_copy_rows_d2h_dma", "rtc_host_register",
    "rtc_host_unregister", "rtc_plan_sim_create", "rtc_plan_sim_launch", "rtc_plan_sim_release", "rtc_frame_loop", "rtc_frame_loop_cameras", "rtc_dma_pending", "rtc_dma_debug_inflight",
    "rtc_probe_ray_triangle", "rtc_probe_ray_sphere", "rtc_probe_environment", "rtc_probe_random",
    "rtc_probe_cluster_bound", "rtc_probe_sun_vanish", "rtc_env_vanish_limit",
]

_lib = None


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def lib() -> C.CDLL:
    """Load librtc.so (built in-tree by `make` / __graft_entry__.build()).  Raises if it is missing:
    there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"librtc.so not built ({LIB_PATH}); run `make` or __graft_entry__.build()")
    # PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, but its libc10_hip links it by file
    # name).  If librtc.so loaded /opt/rocm's copy first, torch would load a second HIP runtime and see no
    # GPU.  Importing torch first makes librtc.so bind to the runtime torch already holds, so device
    # pointers and streams are shared.  Without torch, librtc.so uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp, ip, sz = C.c_void_p, C.c_int, C.c_size_t
    L.rtc_last_error.restype = C.c_char_p
    L.rtc_version.restype = C.c_char_p
    L.rtc_device_count.argtypes = [C.POINTER(C.c_int)]
    L.rtc_load_obj.argtypes = [C.c_char_p, C.POINTER(vp), C.POINTER(C.c_int)]
    L.rtc_parse_triangle_file.argtypes = [C.c_char_p, C.POINTER(vp), C.POINTER(C.c_int)]
    L.rtc_free.argtypes = [vp]
    L.rtc_free.restype = None
    L.rtc_default_spheres.argtypes = [C.POINTER(vp), C.POINTER(C.c_int)]
    L.rtc_default_scene.argtypes = [C.POINTER(Scene)]
    L.rtc_scene_set_sun.argtypes = [C.POINTER(Scene), Vec3]
    L.rtc_camera_basis.argtypes = [Vec3, Vec3, C.c_float, C.POINTER(RtcCamera)]
    L.rtc_write_bmp.argtypes = [C.c_char_p, ip, ip, vp]
    L.rtc_quantize.argtypes = [vp, sz, vp]
    L.rtc_render.argtypes = [vp, ip, vp, ip, C.POINTER(Scene), C.POINTER(RtcCamera), C.POINTER(RtcRenderDesc), ip,
                             vp, vp, C.POINTER(RtcStats)]
    L.rtc_render_multi.argtypes = [vp, ip, vp, ip, C.POINTER(Scene), C.POINTER(RtcCamera),
                                   C.POINTER(RtcRenderDesc), ip, vp, vp, C.POINTER(RtcStats)]
    L.rtc_last_multi_info.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), ip]
    L.rtc_scene_upload.argtypes = [vp, ip, vp, ip, ip, C.POINTER(vp)]
    L.rtc_scene_release.argtypes = [vp]
    L.rtc_scene_kernel_times.argtypes = [vp, vp]
    L.rtc_bounce_hit_share.argtypes = [vp, C.c_int, C.POINTER(C.c_float)]
    L.rtc_scene_chain_wgs.argtypes = [vp]
    L.rtc_scene_set_timing.argtypes = [vp, C.c_int]
    L.rtc_scene_set_geometry_event.argtypes = [vp, vp]
    L.rtc_scene_set_frame_event.argtypes = [vp, vp]
    L.rtc_copy_async.argtypes = [vp, vp, sz, C.c_int, vp]
    L.rtc_copy_d2h_dma.argtypes = [vp, vp, sz]
    L.rtc_copy_rows_d2h_dma.argtypes = [vp, sz, vp, sz, sz, ip]
    L.rtc_host_register.argtypes = [vp, sz]
    L.rtc_host_unregister.argtypes = [vp]
    L.rtc_frame_loop.argtypes = [vp, C.POINTER(Scene), C.POINTER(RtcCamera), C.POINTER(RtcRenderDesc), vp, vp, sz, ip,
                                 ip, vp, C.POINTER(RtcLoopStats)]
    L.rtc_frame_loop_cameras.argtypes = [vp, C.POINTER(Scene), vp, ip, C.POINTER(RtcRenderDesc), vp, vp, sz, ip, ip,
                                         vp, C.POINTER(RtcLoopStats)]
    L.rtc_plan_sim_create.argtypes = [ip, ip, C.POINTER(vp)]
    L.rtc_plan_sim_launch.argtypes = [vp, C.POINTER(RtcRenderDesc), C.c_ulonglong, C.c_ulonglong, C.c_ulonglong, ip, vp,
                                      vp, vp, ip, vp, ip]
    L.rtc_plan_sim_release.argtypes = [vp]
    L.rtc_dma_pending.argtypes = [vp, sz]
    L.rtc_dma_debug_inflight.argtypes = [vp, sz, ip]
    L.rtc_rows_selected.argtypes = [C.POINTER(RtcRenderDesc)]
    L.rtc_render_rows_async.argtypes = [vp, C.POINTER(Scene), C.POINTER(RtcCamera), C.POINTER(RtcRenderDesc), vp, vp,
                                        vp, vp]
    L.rtc_deinterleave_async.argtypes = [vp, ip, ip, ip, ip, vp, vp]
    if hasattr(L, "rtc_deinterleave_bands_async"):  # (absent from round-4 libraries loaded for A/B timing)
        L.rtc_deinterleave_bands_async.argtypes = [vp, ip, ip, ip, ip, ip, vp, vp]
    L.rtc_probe_ray_triangle.argtypes = [vp, vp, sz, vp, vp]
    L.rtc_probe_ray_sphere.argtypes = [vp, vp, sz, vp, vp, vp]
    L.rtc_probe_environment.argtypes = [vp, vp, sz, vp]
    L.rtc_probe_random.argtypes = [vp, sz, ip, vp, vp, vp]
    L.rtc_probe_cluster_bound.argtypes = [vp, ip, vp, sz, vp]
    if hasattr(L, "rtc_probe_sun_vanish"):  # (absent from libraries of earlier rounds loaded for A/B timing)
        L.rtc_probe_sun_vanish.argtypes = [vp, vp, sz, vp, vp]
        L.rtc_env_vanish_limit.argtypes = [vp, vp]
    _lib = L
    return L


class RtcError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib().rtc_last_error().decode(errors="replace")
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


def check(rc: int, where: str) -> None:
    if rc != 0:
        raise RtcError(rc, where)

"""raytracingc_amd -- MI355X-native render path of Atsuyo64/RayTracingC.

The product is librtc.so (HIP kernels for gfx950 behind the C ABI in include/rtc.h).  This package is the
thin host mirror of the reference's interface for that path, with the reference's names:

  scene build   loadOBJTriangles (raytracing.c:100), parseTriangleFile (raytracing.c:76),
                DEFAULT_SPHERES (scene.h:17-19), default_scene (main.c:14,21-28), camera_basis (main.c:252-255)
  render seam   render (main.c:263-304 -> one rtc_render call), render_multi (one process, many GPUs),
                DeviceScene.render_rows_async (device-resident, used by the multi-rank host and bench.py)
  output        vec3ToColor (raytracing.c:11), write_bmp (stbi_write_bmp, main.c:305)
  device probes rayTriangle, raySphere, getEnvironmentLight, RandomValue / RandomValueNormalDistrubtion /
                RandomDiretion -- the renderer's own device functions run on the GPU, for known-answer tests.

There is no CPU fallback: every render call goes to the GPU and raises if librtc.so or the GPU is missing.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._abi import (  # noqa: F401
    CLI_PATH,
    LIB_PATH,
    RAY_DT,
    RTC_F_DEBUG_BOUNCES,
    RTC_F_HOIST_PRIMARY,
    RTC_F_NO_CLUSTER_CULL,
    RTC_F_NO_COOP,
    RTC_F_CHAIN_INLINE,
    RTC_F_OVERLAP,
    RTC_F_HOST_ROWS,
    RTC_F_NO_REORDER,
    RTC_F_NO_TILE_CULL,
    RTC_SEGMENT_COUNTERS,
    RTC_EBUSY,
    RTC_EINVAL,
    RTC_ETIMEDOUT,
    SCENE_DT,
    SPHERE_DT,
    TRIANGLE_DT,
    VEC3_DT,
    EXPORTS,
    Ray,
    RtcCamera,
    RtcError,
    RtcLoopStats,
    RtcRenderDesc,
    RtcStats,
    Scene,
    Vec3,
    check,
    lib,
)
from ._abi import _ptr

__all__ = [
    "loadOBJTriangles", "parseTriangleFile", "default_spheres", "default_scene", "camera_basis", "RenderConfig",
    "render", "render_multi", "DeviceScene", "vec3ToColor", "write_bmp", "rayTriangle", "raySphere",
    "getEnvironmentLight", "random_sequences", "device_count", "lib", "TRIANGLE_DT", "SPHERE_DT", "RAY_DT",
    "SCENE_DT", "RtcError",
]

# main.c:114-116 (camera) and main.c:10-12 (frame) defaults
DEFAULT_ORIGIN = (-4.75, -1.5, -4.75)
DEFAULT_LOOKING_AT = (0.9, -1.2, 1.0)
DEFAULT_FOV = 1.0
DEFAULT_SUN = (-30.0, -85.0, 100.0)


def _take_tris(p: C.c_void_p, n: int) -> np.ndarray:
    out = np.empty(n, dtype=TRIANGLE_DT)
    if n:
        C.memmove(out.ctypes.data, p.value, n * TRIANGLE_DT.itemsize)
    lib().rtc_free(p)
    return out


def loadOBJTriangles(path: str) -> np.ndarray:
    """raytracing.c:100-147 (+ objloader.c): OBJ/MTL -> Triangle[] (x, y negated).  Raises on failure
    (the reference exits 42)."""
    p, n = C.c_void_p(), C.c_int()
    check(lib().rtc_load_obj(path.encode(), C.byref(p), C.byref(n)), "rtc_load_obj")
    return _take_tris(p, n.value)


def parseTriangleFile(path: str) -> np.ndarray:
    """raytracing.c:76-98: triangles.txt -> Triangle[] with counter-clockwise normals."""
    p, n = C.c_void_p(), C.c_int()
    check(lib().rtc_parse_triangle_file(path.encode(), C.byref(p), C.byref(n)), "rtc_parse_triangle_file")
    return _take_tris(p, n.value)


def default_spheres() -> np.ndarray:
    """scene.h:17-19: the single default-mode sphere."""
    p, n = C.c_void_p(), C.c_int()
    check(lib().rtc_default_spheres(C.byref(p), C.byref(n)), "rtc_default_spheres")
    out = np.empty(n.value, dtype=SPHERE_DT)
    C.memmove(out.ctypes.data, p.value, n.value * SPHERE_DT.itemsize)
    return out


def default_scene(sun=DEFAULT_SUN, ground=None, horizon=None, zenith=None, focus=None, intensity=None) -> Scene:
    """main.c:14,21-28 with the CLI overrides of main.c:185-224; the sun is normalised as main.c:247."""
    s = Scene()
    check(lib().rtc_default_scene(C.byref(s)), "rtc_default_scene")
    if ground is not None:
        s.groundColor = Vec3(*ground)
    if horizon is not None:
        s.skyColorHorizon = Vec3(*horizon)
    if zenith is not None:
        s.skyColorZenith = Vec3(*zenith)
    if focus is not None:
        s.sunFocus = focus
    if intensity is not None:
        s.sunIntensity = intensity
    check(lib().rtc_scene_set_sun(C.byref(s), Vec3(*sun)), "rtc_scene_set_sun")
    return s


def camera_basis(origin=DEFAULT_ORIGIN, looking_at=DEFAULT_LOOKING_AT, fov=DEFAULT_FOV) -> RtcCamera:
    """main.c:252-255."""
    cam = RtcCamera()
    check(lib().rtc_camera_basis(Vec3(*origin), Vec3(*looking_at), C.c_float(fov), C.byref(cam)), "rtc_camera_basis")
    return cam


@dataclass
class RenderConfig:
    width: int = 128
    height: int = 128
    spp: int = 4000  # scene.h:26
    max_bounce: int = 10  # main.c:12
    triangles_only: bool = True
    hoist: bool = False
    row_start: int = 0
    row_stride: int = 1
    # rows per interleaved band (rtc.h rowBand): 0/1 single rows y = row_start + k*row_stride; B > 1 (a power of two)
    # bands of B rows starting at row_start + k*row_stride*B
    row_band: int = 0
    debug_bounces: bool = False  # calcDebugColor (raytracing.c:242-260) instead of calcColor
    tile_cull: bool = True  # primary segments visit their 8x8 tile's candidate triangles (bit-exact)
    reorder: bool = True  # dispatch the workgroups that see geometry first (same frame)
    coop: bool = True  # pixels that see geometry: the split launch's rtc_render_chain (same frame)
    cluster_cull: bool = True  # bounce rays skip triangle clusters they provably miss (same frame)
    chain_inline: bool = False  # rtc_render_chain sums each pixel's samples itself (no deferred pass)
    # render_multi: every device copies its rows straight into the host frame instead of the RCCL gather to
    # device 0 (RTC_F_HOST_ROWS; same frame)
    host_rows: bool = False
    # frame pipelining (DeviceScene.render_rows_async): the launch does not join its sky pass into the stream;
    # the frame is complete at the scene's frame event (DeviceScene.set_frame_event); same frame
    overlap: bool = False

    def flags(self) -> int:
        return ((RTC_F_HOIST_PRIMARY if self.hoist else 0) | (RTC_F_DEBUG_BOUNCES if self.debug_bounces else 0)
                | (0 if self.tile_cull else RTC_F_NO_TILE_CULL) | (0 if self.reorder else RTC_F_NO_REORDER)
                | (0 if self.coop else RTC_F_NO_COOP) | (0 if self.cluster_cull else RTC_F_NO_CLUSTER_CULL)
                | (RTC_F_CHAIN_INLINE if self.chain_inline else 0) | (RTC_F_OVERLAP if self.overlap else 0)
                | (RTC_F_HOST_ROWS if self.host_rows else 0))

    def desc(self) -> RtcRenderDesc:
        return RtcRenderDesc(self.width, self.height, self.spp, self.max_bounce, int(self.triangles_only),
                             self.row_start, self.row_stride, self.flags(), self.row_band)

    def rows(self) -> int:
        d = self.desc()
        return lib().rtc_rows_selected(C.byref(d))


def _arr(a, dt):
    if a is None or len(a) == 0:
        return None, 0
    a = np.ascontiguousarray(a, dtype=dt)
    return a, len(a)


def _stats(st: RtcStats) -> dict:
    return {"render_ms": st.renderMs, "frame_ms": st.frameMs, "total_ms": st.totalMs, "segments": st.segments,
            "samples": st.samples, "tri_tests": st.triTests, "cluster_tests": st.clusterTests,
            "discarded_tests": st.discardedTests}


def render(tris, spheres, scene: Scene, cam: RtcCamera, cfg: RenderConfig, device: int = -1,
           want_accum: bool = False):
    """The render seam (main.c:263-304) on one GPU.  Returns (colors uint8 [rows, W, 3],
    accum float32 [rows, W, 3] or None, stats dict)."""
    t, nt = _arr(tris, TRIANGLE_DT)
    s, ns = _arr(spheres, SPHERE_DT)
    rows = cfg.rows()
    colors = np.zeros((rows, cfg.width, 3), np.uint8)
    accum = np.zeros((rows, cfg.width, 3), np.float32) if want_accum else None
    st = RtcStats()
    d = cfg.desc()
    check(lib().rtc_render(_ptr(t), nt, _ptr(s), ns, C.byref(scene), C.byref(cam), C.byref(d), device,
                           _ptr(colors), _ptr(accum), C.byref(st)), "rtc_render")
    return colors, accum, _stats(st)


def render_multi(tris, spheres, scene: Scene, cam: RtcCamera, cfg: RenderConfig, num_devices: int,
                 want_accum: bool = False):
    """Full frame, rows interleaved over `num_devices` GPUs of this process (main.c:84 lifted to GPUs)."""
    t, nt = _arr(tris, TRIANGLE_DT)
    s, ns = _arr(spheres, SPHERE_DT)
    colors = np.zeros((cfg.height, cfg.width, 3), np.uint8)
    accum = np.zeros((cfg.height, cfg.width, 3), np.float32) if want_accum else None
    st = RtcStats()
    d = cfg.desc()
    check(lib().rtc_render_multi(_ptr(t), nt, _ptr(s), ns, C.byref(scene), C.byref(cam), C.byref(d), num_devices,
                                 _ptr(colors), _ptr(accum), C.byref(st)), "rtc_render_multi")
    return colors, accum, _stats(st)


def last_multi_info() -> dict:
    """What this thread's last render_multi ran on (rtc_last_multi_info): path ("none" | "rccl" | "host_rows"), devices,
    and per communicator the rank count RCCL itself reports (ncclCommCount)."""
    path, devs = C.c_int(), C.c_int()
    ranks = (C.c_int * 64)()
    n = lib().rtc_last_multi_info(C.byref(path), C.byref(devs), ranks, 64)
    return {"path": {0: "none", 1: "rccl", 2: "host_rows"}.get(path.value, str(path.value)), "devices": devs.value,
            "comm_ranks": [int(ranks[i]) for i in range(min(n, 64))]}


class DeviceScene:
    """A scene resident in HBM on one device (rtc_scene_upload).  render_rows_async takes raw device
    pointers and a hipStream_t (ints), e.g. from torch tensors / torch.cuda streams."""

    def __init__(self, tris, spheres, device: int = -1):
        t, nt = _arr(tris, TRIANGLE_DT)
        s, ns = _arr(spheres, SPHERE_DT)
        h = C.c_void_p()
        check(lib().rtc_scene_upload(_ptr(t), nt, _ptr(s), ns, device, C.byref(h)), "rtc_scene_upload")
        self._h = h
        self.tri_count = nt
        self.sphere_count = ns

    def render_rows_async(self, scene: Scene, cam: RtcCamera, cfg: RenderConfig, colors_ptr: int,
                          accum_ptr: int | None = None, segments_ptr: int | None = None, stream: int | None = None):
        d = cfg.desc()
        check(lib().rtc_render_rows_async(self._h, C.byref(scene), C.byref(cam), C.byref(d), C.c_void_p(colors_ptr),
                                          C.c_void_p(accum_ptr) if accum_ptr else None,
                                          C.c_void_p(segments_ptr) if segments_ptr else None,
                                          C.c_void_p(stream) if stream else None), "rtc_render_rows_async")

    @property
    def chain_wgs(self) -> int:
        """rtc_render_chain's workgroups per CU for whole frames, chosen at upload (rtc_scene_chain_wgs)."""
        return lib().rtc_scene_chain_wgs(self._h)

    def set_timing(self, enable: bool):
        """Record HIP events around the split launch's kernels from now on (rtc_scene_set_timing)."""
        check(lib().rtc_scene_set_timing(self._h, int(enable)), "rtc_scene_set_timing")

    def set_geometry_event(self, event_handle: int | None):
        """Arm this hipEvent_t (e.g. a torch.cuda.Event's cuda_event) for the NEXT launch only: it records it on its
        stream once the geometry-pixel kernels are enqueued, before the sky pass joins, and forgets it
        (rtc_scene_set_geometry_event, one-shot); None disarms."""
        check(lib().rtc_scene_set_geometry_event(self._h, C.c_void_p(event_handle) if event_handle else None),
              "rtc_scene_set_geometry_event")

    def set_frame_event(self, event_handle: int | None):
        """Arm this hipEvent_t for the NEXT launch only: it records it once its whole frame is written (on its stream
        after the join, or with RenderConfig.overlap on the scene's side stream) and forgets it
        (rtc_scene_set_frame_event, one-shot); None disarms.  A later launch never records it, so releasing the
        event after that launch is safe.  (A torch.cuda.Event has no hipEvent_t before its first record: record
        it once first.)"""
        check(lib().rtc_scene_set_frame_event(self._h, C.c_void_p(event_handle) if event_handle else None),
              "rtc_scene_set_frame_event")

    def frame_loop(self, scene: Scene, cam, cfg: RenderConfig, dev_rows: list, host_rows: list,
                   host_pitch: int, frames: int, stream: int | None = None) -> dict:
        """rtc_frame_loop: `frames` pipelined frames of cfg's rows, rendered into the device buffers dev_rows[k % n]
        and copied (SDMA, native copy thread) into the page-locked host buffers host_rows[k % n] with row pitch
        host_pitch; returns when the last frame is in host memory.  `cam` is one RtcCamera, or a sequence of them:
        frame k then renders with cam[k % len(cam)] (rtc_frame_loop_cameras, a moving camera)."""
        n = len(dev_rows)
        if len(host_rows) != n:
            raise ValueError("frame_loop: one host buffer per device buffer")
        d = cfg.desc()
        dv = (C.c_void_p * n)(*dev_rows)
        hv = (C.c_void_p * n)(*host_rows)
        st = RtcLoopStats()
        strm = C.c_void_p(stream) if stream else None
        if isinstance(cam, RtcCamera):
            check(lib().rtc_frame_loop(self._h, C.byref(scene), C.byref(cam), C.byref(d), dv, hv,
                                       C.c_size_t(host_pitch), n, int(frames), strm, C.byref(st)), "rtc_frame_loop")
        else:
            cams = (RtcCamera * len(cam))(*cam)
            check(lib().rtc_frame_loop_cameras(self._h, C.byref(scene), cams, len(cam), C.byref(d), dv, hv,
                                               C.c_size_t(host_pitch), n, int(frames), strm, C.byref(st)),
                  "rtc_frame_loop_cameras")
        return {"wall_ms": st.wallMs, "frames": st.frames, "enqueue_ms": st.enqueueMs,
                "copy_ms_median": st.copyMsMedian, "copy_ms_max": st.copyMsMax}

    def kernel_times(self):
        """(heavy-tile kernel ms, sky kernel ms) of the last split launch (None if it was not one)."""
        out = (C.c_float * 2)()
        check(lib().rtc_scene_kernel_times(self._h, out), "rtc_scene_kernel_times")
        return None if out[0] < 0 else (float(out[0]), float(out[1]))

    def close(self):
        if self._h:
            lib().rtc_scene_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy_async(dst_ptr: int, src_ptr: int, nbytes: int, blocks: int = 32, stream: int | None = None) -> None:
    """rtc_copy_async: a copy with a small CU footprint (e.g. Color[] into pinned host memory)."""
    check(lib().rtc_copy_async(C.c_void_p(dst_ptr), C.c_void_p(src_ptr), C.c_size_t(nbytes), int(blocks),
                               C.c_void_p(stream) if stream else None), "rtc_copy_async")


def copy_d2h_dma(host_ptr: int, dev_ptr: int, nbytes: int) -> None:
    """rtc_copy_d2h_dma: device -> page-locked host memory on the SDMA engines, blocking (GIL released)."""
    check(lib().rtc_copy_d2h_dma(C.c_void_p(host_ptr), C.c_void_p(dev_ptr), C.c_size_t(nbytes)), "rtc_copy_d2h_dma")


def copy_rows_d2h_dma(host_ptr: int, host_pitch: int, dev_ptr: int, src_pitch: int, row_bytes: int, rows: int) -> None:
    """rtc_copy_rows_d2h_dma: rows of device memory into page-locked host memory with a row pitch (SDMA, blocking):
    a rank's interleaved rows straight into their places of the host frame."""
    check(lib().rtc_copy_rows_d2h_dma(C.c_void_p(host_ptr), C.c_size_t(host_pitch), C.c_void_p(dev_ptr),
                                      C.c_size_t(src_pitch), C.c_size_t(row_bytes), int(rows)), "rtc_copy_rows_d2h_dma")


def host_register(ptr: int, nbytes: int) -> None:
    """rtc_host_register: page-lock an existing host range (e.g. a shared-memory frame every rank maps)."""
    check(lib().rtc_host_register(C.c_void_p(ptr), C.c_size_t(nbytes)), "rtc_host_register")


def host_unregister(ptr: int) -> None:
    """rtc_host_unregister; raises RtcError(RTC_EBUSY) while a timed-out copy may still write the range."""
    check(lib().rtc_host_unregister(C.c_void_p(ptr)), "rtc_host_unregister")


def dma_pending(ptr: int | None = None, nbytes: int = 0) -> int:
    """rtc_dma_pending: copies that timed out (RTC_ETIMEDOUT) and may still read or write [ptr, ptr + nbytes)
    (None: any range).  Buffers they touch must not be freed or reused while this is > 0."""
    n = lib().rtc_dma_pending(C.c_void_p(ptr) if ptr else None, C.c_size_t(nbytes if ptr else 0))
    if n < 0:
        check(n, "rtc_dma_pending")
    return n


def deinterleave_async(compact_ptr: int, parts: int, rows_per_part: int, width: int, height: int, out_ptr: int,
                       stream: int | None = None, row_band: int = 1):
    """rtc_deinterleave_async (single rows) / rtc_deinterleave_bands_async (bands of row_band rows)."""
    if row_band > 1:
        check(lib().rtc_deinterleave_bands_async(C.c_void_p(compact_ptr), parts, rows_per_part, width, height, row_band,
                                                 C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None),
              "rtc_deinterleave_bands_async")
        return
    check(lib().rtc_deinterleave_async(C.c_void_p(compact_ptr), parts, rows_per_part, width, height,
                                       C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None),
          "rtc_deinterleave_async")


def bounce_hit_share(tris) -> float:
    """rtc_bounce_hit_share: the share of diffuse bounce rays from the triangles that hit the scene again (host probe,
    a scheduling hint)."""
    t, nt = _arr(tris, TRIANGLE_DT)
    out = C.c_float()
    check(lib().rtc_bounce_hit_share(_ptr(t), nt, C.byref(out)), "rtc_bounce_hit_share")
    return out.value


def vec3ToColor(accum: np.ndarray) -> np.ndarray:
    """raytracing.c:11-15 / moremath.c:25-30 on a float3 buffer (host)."""
    a = np.ascontiguousarray(accum, dtype=np.float32)
    out = np.empty(a.shape, np.uint8)
    check(lib().rtc_quantize(_ptr(a), a.size // 3, _ptr(out)), "rtc_quantize")
    return out


def write_bmp(path: str, colors: np.ndarray) -> None:
    """stbi_write_bmp(path, W, H, 3, image) (main.c:305)."""
    c = np.ascontiguousarray(colors, dtype=np.uint8)
    h, w = c.shape[0], c.shape[1]
    check(lib().rtc_write_bmp(path.encode(), w, h, _ptr(c)), "rtc_write_bmp")


def device_count() -> int:
    n = C.c_int()
    rc = lib().rtc_device_count(C.byref(n))
    return n.value if rc == 0 else 0


# ---- device probes (same device code as the renderer) --------------------------------------------------
def rayTriangle(rays: np.ndarray, tris: np.ndarray):
    """raytracing.c:186-214 on the GPU, one (ray, triangle) pair per element -> (didHit int32, dst f32)."""
    r = np.ascontiguousarray(rays, RAY_DT)
    t = np.ascontiguousarray(tris, TRIANGLE_DT)
    n = len(r)
    hit, dst = np.zeros(n, np.int32), np.zeros(n, np.float32)
    check(lib().rtc_probe_ray_triangle(_ptr(r), _ptr(t), n, _ptr(hit), _ptr(dst)), "rtc_probe_ray_triangle")
    return hit, dst


def raySphere(rays: np.ndarray, spheres: np.ndarray):
    """raytracing.c:162-184 on the GPU -> (didHit, dst, normal[n,3])."""
    r = np.ascontiguousarray(rays, RAY_DT)
    s = np.ascontiguousarray(spheres, SPHERE_DT)
    n = len(r)
    hit, dst, nrm = np.zeros(n, np.int32), np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    check(lib().rtc_probe_ray_sphere(_ptr(r), _ptr(s), n, _ptr(hit), _ptr(dst), _ptr(nrm)), "rtc_probe_ray_sphere")
    return hit, dst, nrm


def getEnvironmentLight(rays: np.ndarray, scenes: np.ndarray) -> np.ndarray:
    """raytracing.c:151-160 on the GPU -> float32 [n, 3]."""
    r = np.ascontiguousarray(rays, RAY_DT)
    s = np.ascontiguousarray(scenes, SCENE_DT)
    n = len(r)
    out = np.zeros((n, 3), np.float32)
    check(lib().rtc_probe_environment(_ptr(r), _ptr(s), n, _ptr(out)), "rtc_probe_environment")
    return out


def sun_vanish_probe(rays: np.ndarray, scenes: np.ndarray):
    """The sky kernel's per-pixel sun skip on the GPU: (vanish int32 [n], environment float32 [n, 3] evaluated with it)."""
    r = np.ascontiguousarray(rays, RAY_DT)
    s = np.ascontiguousarray(scenes, SCENE_DT)
    n = len(r)
    v = np.zeros(n, np.int32)
    out = np.zeros((n, 3), np.float32)
    check(lib().rtc_probe_sun_vanish(_ptr(r), _ptr(s), n, _ptr(v), _ptr(out)), "rtc_probe_sun_vanish")
    return v, out


def env_vanish_limit(scene) -> float:
    """The bound on focus * log2(x) below which the sky kernel skips the sun term (host only; -inf: never)."""
    s = np.ascontiguousarray(scene, SCENE_DT).reshape(1)
    out = C.c_double(0.0)
    check(lib().rtc_env_vanish_limit(_ptr(s), C.byref(out)), "rtc_env_vanish_limit")
    return out.value


def random_sequences(seeds: np.ndarray, draws: int):
    """moremath.c:89-108 on the GPU: per seed, `draws` x RandomValue, x RandomValueNormalDistrubtion and
    x RandomDiretion, each sequence restarted from the seed."""
    sd = np.ascontiguousarray(seeds, np.uint32)
    n = len(sd)
    u = np.zeros((n, draws), np.float32)
    g = np.zeros((n, draws), np.float32)
    d = np.zeros((n, draws, 3), np.float32)
    check(lib().rtc_probe_random(_ptr(sd), n, draws, _ptr(u), _ptr(g), _ptr(d)), "rtc_probe_random")
    return u, g, d


def cluster_bound_probe(tris: np.ndarray, rays: np.ndarray) -> dict:
    """Soundness of the bounce-ray cluster culling on the GPU (rtc_probe_cluster_bound): hits inside culled
    clusters (must be 0), clusters culled, cluster tests, hits, largest hit excess over a bounding radius; hits
    on triangles the first-bounce reach mask calls unreachable from the ray's origin (must be 0), pairs so called."""
    t = np.ascontiguousarray(tris, TRIANGLE_DT)
    r = np.ascontiguousarray(rays, RAY_DT)
    c = np.zeros(7, np.uint64)
    check(lib().rtc_probe_cluster_bound(_ptr(t), len(t), _ptr(r), len(r), _ptr(c)), "rtc_probe_cluster_bound")
    return {"violations": int(c[0]), "culled": int(c[1]), "tests": int(c[2]), "hits": int(c[3]),
            "max_excess": float(np.array([c[4]], np.uint64).astype(np.uint32).view(np.float32)[0]),
            "reach_violations": int(c[5]), "unreachable": int(c[6])}

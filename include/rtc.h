/*
 * rtc.h -- C ABI of the MI355X-native render path (librtc.so).
 *
 * This is the drop-in boundary for the reference's render seam, main.c:263-304 (the pthread fan-out of
 * rowThread, main.c:81-104, over calcColor raytracing.c:262-296).  The reference has no plugin or FFI API;
 * its only "interface" for this path is that seam plus the scene-build / output functions either side
 * of it, so the entry points below are what a maintainer binds in place of that region.
 *
 * Plain C: plain pointers and sizes, no torch or HIP types.  All structs keep the reference's byte
 * layouts (raytracing.h:7-69, moremath.h:10-13) so host arrays produced by the reference's own loaders
 * pass through unconverted.
 *
 * Error convention: 0 = OK; a negative value is either -(hipError_t) (|v| < 10000) or one of the RTC_E*
 * codes below; a positive value is an RCCL ncclResult_t (rtc_render_multi).  Nothing here calls exit();
 * rtc_last_error() returns a message for the calling thread.  Entry points that select a device restore
 * the caller's current device before returning.
 */
#ifndef RTC_H
#define RTC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference types (identical layouts; sizes are static_assert-ed in the implementation) ------------ */
typedef unsigned char uint8;                                                   /* moremath.h:6 */
typedef struct vec3 { float x, y, z; } vec3;                                   /* moremath.h:10-13, 12 B */
typedef struct Scene {                                                         /* raytracing.h:7-11, 56 B */
    vec3 normalizedSunDirection, skyColorHorizon, skyColorZenith, groundColor;
    float sunFocus, sunIntensity;
} Scene;
typedef struct Color { uint8 r, g, b; } Color;                                 /* raytracing.h:15-18, 3 B */
typedef struct Material { vec3 color; float emissionStrength; float smoothness; } Material; /* :25-30, 20 B */
typedef struct Sphere { vec3 pos; float r; Material mat; } Sphere;             /* raytracing.h:34-39, 36 B */
typedef struct Triangle { vec3 posA, posB, posC, normal; Material mat; } Triangle; /* :41-45, 68 B */
typedef struct Ray { vec3 pos; vec3 dir; } Ray;                                /* raytracing.h:64-68, 24 B */

/* ---- render description ---------------------------------------------------------------------------- */
/* Camera: origin plus the basis main.c:252-255 computes, and fov (main.c:116). */
typedef struct RtcCamera { vec3 origin, ex, ey, ez; float fov; } RtcCamera;   /* 52 B */

/* Which pixels and how.  width/height/maxBounce = main.c:10-12; spp = accumulationCount (scene.h:26);
 * trianglesOnly = main.c:113,241.  Rows rendered: y = rowStart + k*rowStride for k = 0..ceil(..)-1, the
 * reference's row interleave (main.c:84) lifted to devices/ranks.  rowStride = 1, rowStart = 0 renders the
 * whole frame.  rowBand = B > 1 (a power of two, at most 64; 0 or 1: single rows) interleaves bands of B rows
 * instead: launch row r is image row y = rowStart + (r / B)*rowStride*B + r % B -- rank g of G renders the bands
 * b = g, g + G, ... with rowStart = g*B, rowStride = G (north_star's row-tile split: with B = 8 a rank's 8x8 pixel
 * tiles are 8 adjacent image rows, not 8 rows G apart).  The launch writes its rows compactly in that order.  The
 * frame does not depend on the partition (the seed is the absolute pixel index, main.c:95). */
typedef struct RtcRenderDesc {
    int width, height;
    int spp;
    int maxBounce;
    int trianglesOnly;
    int rowStart, rowStride;
    int flags;                 /* RTC_F_* */
    int rowBand;               /* rows per interleaved band (0 or 1: single rows) */
} RtcRenderDesc;

#define RTC_F_HOIST_PRIMARY 0x1  /* bit-exact: trace each pixel's primary ray once; default off */
#define RTC_F_DEBUG_BOUNCES 0x2  /* calcDebugColor (raytracing.c:242-260) instead of calcColor: bounce-count grey */
#define RTC_F_NO_TILE_CULL  0x4  /* primary segments test every triangle (brute force, as calculateRayCollision
                                    does) instead of the 8x8 tile's candidate list; same output bit for bit */
#define RTC_F_NO_REORDER    0x8  /* dispatch workgroups in raster order instead of heaviest first (for A/B
                                    timing; the frame is identical) */
#define RTC_F_NO_COOP       0x10 /* pixels that see geometry are rendered like the rest, one lane per pixel
                                    (rtc_render_kernel), instead of by the split launch's rtc_render_chain
                                    (A/B timing; the frame is identical) */
#define RTC_F_NO_CLUSTER_CULL 0x20 /* bounce rays test every triangle instead of only the clusters their
                                      half-line may reach (A/B timing; identical frame) */
/* The split launch renders the pixels that see geometry with rtc_render_chain (state-indexed samples: lanes
 * evaluate the samples that start at consecutive RNG offsets, then the chain of the reference's samples is walked
 * in order).  0x40, 0x80, 0x100 and 0x200 selected older kernels for A/B timing; they were removed and these flags
 * are now RTC_EINVAL. */
#define RTC_F_COOP4         0x40 /* removed: RTC_EINVAL */
#define RTC_F_COOP8         0x80 /* removed: RTC_EINVAL */
#define RTC_F_PIPE          0x200 /* removed: RTC_EINVAL */
#define RTC_F_SPEC          0x100 /* removed: RTC_EINVAL */
#define RTC_F_CHAIN_INLINE  0x400 /* rtc_render_chain adds each pixel's samples itself instead of deferring the
                                     in-order sum to a separate pass (identical frame; the default for a small share
                                     of a row-partitioned frame, rowStride > 1 and width * rows <= 600,000, and for
                                     the overlapped launches on the alternating streams, RTC_F_OVERLAP) */
#define RTC_F_HOST_ROWS     0x1000 /* rtc_render_multi only: no gather -- every device copies its rows straight into
                                      their places of the host frame (rtc_copy_rows_d2h_dma, its own PCIe link);
                                      without it the parts are gathered to device 0 over RCCL, re-interleaved there
                                      and copied once.  Same frame bit for bit. */
#define RTC_F_OVERLAP       0x800 /* frame pipelining (device-resident split only): the launch does not make
                                     `stream` wait for its sky pass, so the next launches on the same scene render
                                     (scratch in 8 slots) while this one's sky pass still runs.  A later overlapped
                                     launch waits for it only when it would rewrite its scratch slot (8 launches
                                     later) or writes the same Color / accumulator buffer with other rows, camera or
                                     environment; a later launch that is not overlapped waits for it before its
                                     first kernel.  Every overlapped launch but a row-stride-1 frame of at most
                                     600 k pixels prepares, culls and runs its geometry kernel on one of two scene
                                     streams (alternating), unordered against the previous launch's geometry
                                     kernel, and sums each pixel's samples in-kernel: such a launch starts after
                                     everything enqueued on `stream` before it, but `stream` is not made to wait for
                                     its kernels.  Every overlapped launch's frame is complete when the scene's frame
                                     event (rtc_scene_set_frame_event) fires -- consume it there, not at `stream`;
                                     with segment counters requested the launch joins as usual.  Same frame bit for
                                     bit. */

typedef struct RtcStats {
    double renderMs;             /* device time of the render launch (slowest device), HIP events */
    double totalMs;              /* wall time of the whole call incl. scene upload, allocations, readback */
    unsigned long long segments; /* closest-hit queries traced (calculateRayCollision calls) */
    unsigned long long samples;  /* camera samples = pixels * spp */
    unsigned long long triTests; /* ray-triangle tests evaluated (segments x triangles the segment visits) */
    unsigned long long clusterTests; /* ray-cluster bounding-ball tests (cooperative path, bounce rays) */
    unsigned long long discardedTests; /* ray-triangle tests of speculative samples not accumulated */
    double frameMs;              /* SURVEY.md §8(d) frame time: first render kernel launch after the scene upload
                                    until Color[W*H] is in (pinned) host memory -- render, RCCL gather and
                                    re-interleave (multi), D2H; HIP events on device 0 */
} RtcStats;

/* ---- error codes ----------------------------------------------------------------------------------- */
#define RTC_OK 0
#define RTC_EINVAL (-10001)
#define RTC_ENODEV (-10002)
#define RTC_EIO (-10003)
#define RTC_ENOMEM (-10004)
#define RTC_EFORMAT (-10005)
#define RTC_ETIMEDOUT (-10006) /* an SDMA copy did not complete in time and may still run (rtc_dma_pending) */
#define RTC_EBUSY (-10007)     /* a range a timed-out copy may still write (rtc_host_unregister) */

const char *rtc_last_error(void);
const char *rtc_version(void);
int rtc_device_count(int *count);

/* ---- scene build (host; restates objloader.c:340-551 + raytracing.c:19-147) ------------------------ */
/* loadOBJTriangles (raytracing.c:100-147): OBJ/MTL -> Triangle[] with the x,y negation.  On failure
 * returns RTC_EIO (the reference exits 42, raytracing.c:106-110; the CLI driver keeps that). *outTris is
 * malloc'd; free with rtc_free. */
int rtc_load_obj(const char *path, Triangle **outTris, int *outCount);
/* parseTriangleFile (raytracing.c:76-98) incl. cleanFile (:47-74).  Writes "<path>.parsed" beside the
 * input exactly like the reference.  Missing file -> RTC_EIO with count 0 (the reference silently keeps 0). */
int rtc_parse_triangle_file(const char *path, Triangle **outTris, int *outCount);
void rtc_free(void *p);
/* The default scene's sphere list (scene.h:17-19) and sky/sun (main.c:14,21-28), sun normalised as main.c:247. */
int rtc_default_spheres(const Sphere **outSpheres, int *outCount);
int rtc_default_scene(Scene *outScene);
int rtc_scene_set_sun(Scene *scene, vec3 sunDirection);
/* main.c:252-255 */
int rtc_camera_basis(vec3 origin, vec3 lookingAt, float fov, RtcCamera *outCam);
/* 24-bit BMP, byte-identical to stbi_write_bmp (stbi_image_write.h:492-529) */
int rtc_write_bmp(const char *path, int width, int height, const Color *image);
/* vec3ToColor / floatToUint (raytracing.c:11-15, moremath.c:25-30) on a host float3 buffer */
int rtc_quantize(const float *accum, size_t pixels, Color *out);

/* ---- render: host buffers (the seam main.c:263-304) ------------------------------------------------ */
/* Uploads the scene to HBM, renders the rows selected by d (normally the full frame) on `device`
 * (-1 = current), writes Color rows (row-major, y = 0 top; a partial row set is written compactly in
 * row order) and optionally the pre-quantisation float3 accumulator.  Inputs are borrowed for the call. */
int rtc_render(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
               const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int device,
               Color *outImage, float *outAccum, RtcStats *stats);

/* Single-process multi-GPU variant of rtc_render (replaces the 12-pthread fan-out main.c:285-302): devices
 * 0..numDevices-1 each render the rows y = g + k*numDevices (the reference's row interleave, main.c:84,
 * lifted to GPUs) -- or, with d->rowBand = B > 1, the bands of B rows b = g + k*numDevices -- into a compact part,
 * concurrently; one RCCL communicator clique (ncclCommInitAll) gathers
 * the parts to device 0 over xGMI (ncclGather, grouped), device 0 re-interleaves them and one D2H brings the
 * frame to the host.  Output is bit-identical to numDevices = 1 (the seed is the absolute pixel index,
 * main.c:95).  RCCL errors are returned as positive ncclResult_t values.  stats->renderMs = slowest
 * device's render launch; stats->frameMs = render + gather + re-interleave + D2H. */
int rtc_render_multi(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                     const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int numDevices,
                     Color *outImage, float *outAccum, RtcStats *stats);
/* What the calling thread's last rtc_render_multi ran on: *path 0 (no call yet), 1 (RCCL gather) or 2 (RTC_F_HOST_ROWS,
 * no communicator); *devices its numDevices; commRanks[g] (up to maxComms) the rank count communicator g reports itself
 * (ncclCommCount; -1 if not reported).  Returns the number of communicators.  No reference counterpart: it shows that
 * RCCL saw the whole clique (main.c:285-302's fan-out lifted to GPUs). */
int rtc_last_multi_info(int *path, int *devices, int *commRanks, int maxComms);

/* ---- render: device-resident (used by the multi-GPU host and bench) -------------------------------- */
typedef struct RtcDeviceScene RtcDeviceScene;
int rtc_scene_upload(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                     int device, RtcDeviceScene **out);
int rtc_scene_release(RtcDeviceScene *s);
/* Number of rows d selects (ceil((height - rowStart) / rowStride) for single rows; with bands, the full bands' rows
 * plus the last band's rows inside the frame), 0 if none. */
int rtc_rows_selected(const RtcRenderDesc *d);
/* Asynchronous on `stream` (a hipStream_t, NULL = default stream).  dColors: device buffer of
 * rows_selected*width*3 bytes; dAccum: nullable device float buffer rows_selected*width*3; dSegments:
 * nullable device u64[RTC_SEGMENT_COUNTERS] the kernel atomically adds to: [0] calculateRayCollision calls
 * (the reference's segment count), [1] closest-hit queries actually traced (smaller with
 * RTC_F_HOIST_PRIMARY), [2] ray-triangle tests of the accumulated samples, [3] ray-cluster bounding-ball
 * tests, [4] ray-triangle tests of speculatively evaluated samples that were not accumulated (state-indexed
 * window lanes off the chain, mispredicted speculative samples); [2] + [4] = every test evaluated.
 * A scene handle serves one stream at a time: its per-launch scratch (primary-ray records, tile candidate
 * lists) is rewritten by every launch. */
#define RTC_SEGMENT_COUNTERS 5
/* Per-kernel timing of the split launch: with rtc_scene_set_timing(s, 1) every later launch on s records HIP
 * events around its two kernels (off by default: the records cost each launch a few microseconds), and
 * rtc_scene_kernel_times returns the device times (ms) of the last launch: out[0] the geometry-pixel kernel
 * (rtc_render_chain by default, without the rtc_accumulate_samples pass that follows it), out[1] the sky
 * kernel (concurrent, on the scene's side stream); -1 when that launch recorded none.  Waits for that launch
 * to finish. */
int rtc_scene_set_timing(RtcDeviceScene *s, int enable);
/* Pipelining hooks.  Both are ONE-SHOT: the event is armed for the next launch on s that renders rows
 * (rtc_render_rows_async with rows_selected > 0), which records it and forgets it, so no later launch can record
 * an event its caller has released.  Arm again before every launch that should record one; NULL disarms.
 * Geometry event: recorded on the launch's stream once the geometry-pixel kernels are enqueued, before the join
 * with the sky pass; a caller can start the previous frame's D2H there, so that the copy overlaps the sky pass
 * instead of the next frame's persistent geometry kernel (whose workgroups then all start at once). */
int rtc_scene_set_geometry_event(RtcDeviceScene *s, void *event);
/* Frame event: recorded once the whole frame -- the geometry pixels and the sky pass -- is written: on the launch's
 * stream after the join, or with RTC_F_OVERLAP (no join) on the scene's side stream after both passes.  Consumers
 * of the frame (a D2H, a gather) wait for it.  The event must stay valid until that launch has been enqueued
 * (rtc_render_rows_async returned). */
int rtc_scene_set_frame_event(RtcDeviceScene *s, void *event);
int rtc_scene_kernel_times(const RtcDeviceScene *s, float out[2]);
/* Scheduling hints chosen at upload (no reference counterpart; they never change a frame):
 * rtc_bounce_hit_share estimates (host only, fixed-seed probe) the share of diffuse bounce rays from the triangles that
 * hit the scene again; rtc_scene_chain_wgs reports the geometry kernel's workgroups per CU for whole frames that the
 * scene got from it (4 above 0.15, else 3; small row shares run 3). */
int rtc_bounce_hit_share(const Triangle *tris, int triCount, float *share);
int rtc_scene_chain_wgs(const RtcDeviceScene *s);
int rtc_render_rows_async(const RtcDeviceScene *s, const Scene *scene, const RtcCamera *cam,
                          const RtcRenderDesc *d, void *dColors, float *dAccum,
                          unsigned long long *dSegments, void *stream);
/* Copy `bytes` (16-byte aligned pointers) on `stream` with `blocks` workgroups (<= 0: 32): e.g. Color[] from HBM
 * into pinned host memory with a small CU footprint while render kernels run (the runtime's D2H blit kernel
 * takes one workgroup on every CU).  Asynchronous. */
int rtc_copy_async(void *dst, const void *src, size_t bytes, int blocks, void *stream);
/* Copy `bytes` of device memory into page-locked host memory (hipHostMalloc) with the SDMA copy engines (HSA
 * runtime), blocking until done; the caller orders it after the frame (e.g. a host thread that waits for the
 * frame's event first).  Unlike the runtime's D2H blit kernel it does not slow render kernels running at the
 * same time (~0.01 vs ~0.1 ms per 1080p frame). */
int rtc_copy_d2h_dma(void *hostDst, const void *devSrc, size_t bytes);
/* Copy-engine timeouts (rtc_copy_d2h_dma, rtc_copy_rows_d2h_dma, rtc_frame_loop): a copy that has not completed after
 * 20 s (RTC_DMA_TIMEOUT_MS overrides) returns RTC_ETIMEDOUT, but the engine may still read its source and write its
 * destination.  The library keeps such a copy listed (its completion signal is neither reused nor destroyed) until the
 * signal shows it ended.  After RTC_ETIMEDOUT the caller must not free, reuse or unregister either buffer while
 * rtc_dma_pending over it is > 0; rtc_host_unregister refuses such a range with RTC_EBUSY.
 * rtc_dma_pending: the number of listed copies whose source or destination overlaps [p, p + bytes) (p = NULL: all),
 * reaping those that have ended. */
int rtc_dma_pending(const void *p, size_t bytes);
/* Test hook of that bookkeeping (no copy engine involved): list (pending != 0) or drop a simulated in-flight copy
 * into [p, p + bytes). */
int rtc_dma_debug_inflight(void *p, size_t bytes, int pending);
/* Copy `rows` rows of `rowBytes` from device memory (row pitch srcPitch) into page-locked host memory (row pitch
 * hostPitch) with the SDMA engines, blocking until done: one SDMA sub-window copy (all pointers, pitches and rowBytes
 * multiples of 4), else one linear copy per row.  A rank's compact rows y = r + k*G (rtc_render_rows_async with
 * rowStart r, rowStride G) land in their places of the interleaved host frame with hostDst = frame + r*W*3 and
 * hostPitch = G*W*3 -- every GPU writes its own rows over its own PCIe link, as the reference's threads write their
 * rows into the shared image (main.c:84, :285-302).  The host memory is hipHostMalloc'd or registered
 * (rtc_host_register, e.g. a shared-memory frame all ranks map); the copy runs through the CPU agent nearest the
 * source GPU. */
int rtc_copy_rows_d2h_dma(void *hostDst, size_t hostPitch, const void *devSrc, size_t srcPitch, size_t rowBytes,
                          int rows);
/* Page-lock (hsa_amd_memory_lock, every agent) / release an existing host range so the copies above can target it. */
int rtc_host_register(void *p, size_t bytes);
int rtc_host_unregister(void *p);

/* Test hooks of the launch planner (rtc_plan.h; no GPU involved): the ordering decisions rtc_render_rows_async would take
 * for a sequence of launches on a scene of triCount triangles, without any device.  rtc_plan_sim_launch plans one launch
 * (d; the caller's stream identity `stream`, 0 = the null stream; Color / accumulator buffer identities; segment counters
 * asked for or not; the camera cam[13] = origin, ex, ey, ez, fov and environment env[14] = sun, horizon, zenith, ground,
 * focus, intensity that decide the pixel values) and writes its operations as 4 ints each (kind 0 kernel / 1 record /
 * 2 wait, stream 0 caller / 1, 2 cull streams / 3 side stream, event, kernel) and each kernel's memory footprint as 6 u64
 * each (op index, resource, access, id, byte range), then one u64 record (~0, scratch regrown, slot, alternating streams,
 * overlapped, slot offset).  Returns nOps | (footprint records << 8).  legacySlotLayout: round 5's broken scratch
 * layout (slot h at h x the launch's own slot size), for the test that must catch it. */
typedef struct RtcPlanSim RtcPlanSim;
int rtc_plan_sim_create(int triCount, int legacySlotLayout, RtcPlanSim **out);
int rtc_plan_sim_launch(RtcPlanSim *sim, const RtcRenderDesc *d, unsigned long long stream, unsigned long long colors,
                        unsigned long long accum, int segments, const float cam[13], const float env[14], int *ops,
                        int maxOps, unsigned long long *footprint, int maxFootprint);
int rtc_plan_sim_release(RtcPlanSim *sim);

/* Pipelined frames on one device, driven from native code (the per-frame host cost is the launch enqueue alone).
 * Frame k renders d's rows with RTC_F_OVERLAP into devRows[k % nbuf] (device buffers of rows_selected*width*3 bytes)
 * on `stream`; a copy thread waits for the frame's event and moves the rows into hostRows[k % nbuf] (page-locked,
 * pitch hostPitch between consecutive rows, or between consecutive bands of d->rowBand rows, each band's rows
 * adjacent) with rtc_copy_rows_d2h_dma; buffer b is rendered into again once its copy has finished.
 * Returns when the last frame's rows are in host memory.  Uses the scene's frame event hook itself. */
typedef struct RtcLoopStats {
    double wallMs;       /* first enqueue .. the last frame's rows in host memory (host clock) */
    int frames;
    double enqueueMs;    /* host time spent in rtc_render_rows_async, summed over the frames */
    double copyMsMedian; /* one frame's SDMA copy as the copy thread timed it: median and maximum */
    double copyMsMax;
} RtcLoopStats;
int rtc_frame_loop(RtcDeviceScene *s, const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d,
                   void *const *devRows, void *const *hostRows, size_t hostPitch, int nbuf, int frames, void *stream,
                   RtcLoopStats *stats);
/* The same loop with a moving camera: frame k renders with cams[k % ncams] (e.g. an orbit; every camera change
 * re-derives the per-launch primary records, and an unjoined sky pass of another camera is waited for before the
 * next launch writes its buffer).  rtc_frame_loop is this with ncams = 1.  On an error (e.g. RTC_ETIMEDOUT from a
 * copy) the loop stops enqueueing, waits for the copies it started and returns the first error; no buffer is
 * rendered into again after its copy failed. */
int rtc_frame_loop_cameras(RtcDeviceScene *s, const Scene *scene, const RtcCamera *cams, int ncams,
                           const RtcRenderDesc *d, void *const *devRows, void *const *hostRows, size_t hostPitch,
                           int nbuf, int frames, void *stream, RtcLoopStats *stats);

/* Re-assemble a row-interleaved gather: dCompact holds `parts` blocks of rowsPerPart*width*3 bytes, block
 * g holding rows y = g + k*parts; dOut receives the height*width*3 frame.  Asynchronous on `stream`. */
int rtc_deinterleave_async(const void *dCompact, int parts, int rowsPerPart, int width, int height,
                           void *dOut, void *stream);
/* The same for parts of interleaved bands of rowBand rows (RtcRenderDesc.rowBand; 0 or 1: single rows): block g holds
 * the bands b = g, g + parts, ... (rows b*rowBand .. b*rowBand + rowBand - 1), each band's rows in order. */
int rtc_deinterleave_bands_async(const void *dCompact, int parts, int rowsPerPart, int width, int height, int rowBand,
                                 void *dOut, void *stream);

/* ---- device probes: run single reference functions on the GPU for known-answer tests --------------- */
/* Each copies inputs to the current device, runs one kernel of the same device code the renderer uses,
 * and copies results back (synchronous). */
int rtc_probe_ray_triangle(const Ray *rays, const Triangle *tris, size_t n, int *didHit, float *dst);   /* raytracing.c:186 */
int rtc_probe_ray_sphere(const Ray *rays, const Sphere *spheres, size_t n, int *didHit, float *dst,
                         vec3 *normal);                                                                 /* raytracing.c:162 */
int rtc_probe_environment(const Ray *rays, const Scene *scenes, size_t n, vec3 *out);                  /* raytracing.c:151 */
int rtc_probe_random(const unsigned int *seeds, size_t n, int draws, float *uniform, float *normal,
                     vec3 *direction);                                                                  /* moremath.c:89-108 */
/* The sky kernel's per-pixel sun skip (no reference counterpart; raytracing.c:155-158 is what it must reproduce): vanish[i]
 * = 1 where the sun term is proved below half an ulp of every colour component, and out[i] = getEnvironmentLight
 * evaluated with that skip (equal to rtc_probe_environment's value for every ray). */
int rtc_probe_sun_vanish(const Ray *rays, const Scene *scenes, size_t n, int *vanish, vec3 *out);
/* The bound the skip compares focus * log2(x) with (host only; -inf: the scene's colours or sun admit no skip). */
int rtc_env_vanish_limit(const Scene *scene, double *limit);
/* Soundness probe of the bounce-ray cluster culling (no reference counterpart; raytracing.c:186-214 is the
 * per-triangle test it must never contradict): clusters `tris` as rtc_scene_upload does and, for every ray and
 * every cluster ball (8 triangles) and chunk ball (32 clusters, scenes of more than one chunk), counts [0] hits
 * inside balls the ray was culled from (0 when sound), [1] balls culled, [2] ball tests, [3] hits, [4] float
 * bits of the largest hit-point excess over a ball's radius, [5] hits on triangles the first-bounce reach mask
 * calls unreachable from the ray's origin (0 when sound), [6] (ray, triangle) pairs it calls so. */
int rtc_probe_cluster_bound(const Triangle *tris, int triCount, const Ray *rays, size_t n,
                            unsigned long long counts[7]);

#ifdef __cplusplus
}
#endif
#endif /* RTC_H */

/*
 * rtc_render.hip -- the MI355X render path behind include/rtc.h.
 *
 * Replaces the reference's render region main.c:263-304: rowThread (main.c:81-104) fanned out over 12
 * pthreads, each pixel running accumulationCount x calcColor (raytracing.c:262-296) over a brute-force
 * calculateRayCollision (raytracing.c:216-240).
 *
 * Design:
 *  - one lane per pixel, a 256-thread workgroup = 16x16 pixels, each wave an 8x8 tile (coherent primary
 *    rays for the wave-uniform early-outs);
 *  - each lane runs its pixel's samples sequentially (the RNG state x + y*W advances across samples,
 *    main.c:95, so samples of one pixel cannot be split) as a segment state machine: every iteration of
 *    the wave loop is ONE closest-hit query for every live lane, so the triangle loop is always
 *    wave-uniform and triangles are read with scalar loads (SGPR operands, no LDS/VGPR traffic);
 *  - triangles are stored with the edges AB, AC precomputed (bit-exact: the same f32 subtraction);
 *  - quantisation (vec3ToColor) is fused; the float accumulator is written only when asked for.
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifdef RTC_DIAG
__device__ unsigned g_rtc_bmfall[65536]; /* Box-Muller exact fallbacks per wave slot (diagnostic builds) */
#endif

#include "../../include/rtc.h"
#include "rtc_layout.h"
#include "rtc_internal.h"
#include "rtc_hip_util.h"

static_assert(sizeof(vec3) == 12, "vec3 layout");
static_assert(sizeof(Material) == 20, "Material layout");
static_assert(sizeof(Sphere) == 36, "Sphere layout");
static_assert(sizeof(Triangle) == 68, "Triangle layout");
static_assert(sizeof(Scene) == 56, "Scene layout");
static_assert(sizeof(Color) == 3, "Color layout");
static_assert(sizeof(Ray) == 24, "Ray layout");
static_assert(sizeof(RtcRenderDesc) == 36, "RtcRenderDesc layout (ctypes mirror: raytracingc_amd/_abi.py)");

using namespace rtcdev;

/* ---- errors ---------------------------------------------------------------------------------------- */
static thread_local char g_err[1024] = "";

extern "C" int rtc_fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" void rtc_log(int level, const char *fmt, ...)
{
    const char *v = getenv("RTC_VERBOSE");
    if (!v || atoi(v) < level)
        return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
}

extern "C" const char *rtc_last_error(void) { return g_err; }
extern "C" const char *rtc_version(void) { return "rtc-mi355x 0.1 (gfx950)"; }


extern "C" int rtc_device_count(int *count)
{
    if (!count)
        return rtc_fail(RTC_EINVAL, "null count");
    *count = 0;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return rtc_fail(RTC_ENODEV, "no HIP device: %s", hipGetErrorString(e));
    *count = n;
    return 0;
}

/* ---- device scene layout: rtc_layout.h; upload: rtc_scene.hip; probes: rtc_probe.hip ---------------------- */
constexpr int kUnroll = 2; /* records per scalar-load batch; arrays are padded to a multiple of 8 */
static_assert(8 % (2 * kUnroll) == 0 || kUnroll == 1, "padding assumes two batches divide 8");

/* ---- the render kernel ---------------------------------------------------------------------------- */
/* one deferred sample: radiance * (1/spp), 12 B (stored and read as 3 dwords) */
struct SampleSlot {
    float x, y, z;
};

struct RenderParams {
    const DevTri *__restrict__ tris;
    const DevMat *__restrict__ mats;
    const DevSphere *__restrict__ spheres;
    const DevPrimF *__restrict__ primF;
    const DevPrimX *__restrict__ primX;
    const DevTri *__restrict__ clTris;         /* cluster order (rtc_build_clusters) */
    const DevCluster *__restrict__ clusters;
    const DevCluster *__restrict__ chunks;
    int chunkCount;
    int clusterCount, clusterCull;
    const unsigned long long *__restrict__ tileMask; /* null: primary segments test every triangle */
    const unsigned long long *__restrict__ pixMask;  /* per 8x8 tile: pixels with a primary candidate (bit i =
                                                       pixel i, row-major); the others see only the sky */
    const int *__restrict__ order; /* null: identity; else launch slot -> workgroup (heavy first) */
    /* rtc_super_cull's survivors (maskWords u64 per superblock of kSuperBlocks x kSuperBlocks workgroup blocks,
     * superX per row of superblocks); null: rtc_tile_cull tests every triangle at level 1 */
    const unsigned long long *__restrict__ superMask;
    int superX;
    /* rtc_render_chain's work: kGeoLists sub-lists of geometry pixels (tile*64 + bit), filled by rtc_tile_cull
     * (tile t appends to sub-list t % kGeoLists, one atomic per tile with geometry, spread over kGeoLists
     * counters in separate cache lines); geoCount[l * 32] = entries of sub-list l, zeroed by the previous split
     * launch's rtc_tile_cull on the same stream, or by rtc_prep_primary */
    int *__restrict__ geoCount;
    int *__restrict__ geoCountNext; /* the next split launch's counters, zeroed by this launch's rtc_tile_cull */
    int *__restrict__ geoList;
    int geoCap; /* entries per sub-list */
    int cullPrio; /* rtc_tile_cull's waves at issue priority 3 (kCullPrioMinPixels) */
    int blocksX; /* 16x16 blocks per row of the launch */
    /* merged sky pass (rtcplan::Plan::merge; null: none): rtc_tile_cull writes each geometry pixel's item (pixItem[tile * 64
     * + bit]), rtc_render_chain each item's Color bytes (geoColor[item], bytes 0-2), and the sky pass -- after it -- every
     * pixel's Color in whole lines */
    unsigned *__restrict__ pixItem;
    unsigned *__restrict__ geoColor;
    SampleSlot *__restrict__ sampleBuf; /* rtc_render_chain, deferred accumulation: [item][spp] radiance * (1/spp) */
    int *__restrict__ itemPix;      /* [item] the pixel's offset in the launch's Color rows */
    int sampleCap;                  /* items with a slot in sampleBuf; items beyond it accumulate in-kernel */
    int chainPrimF;                 /* rtc_render_chain stages DevPrimF[triPadded] in LDS */
    unsigned char *__restrict__ colors;
    float *__restrict__ accum;
    unsigned long long *__restrict__ segments; /* [0] calculateRayCollision calls, [1] traced, [2] tri tests */
    unsigned long long *__restrict__ segSlots; /* kSegSlots x kSegSlotStride partial counters (flush_counters) */
    int triCount, triPadded, sphereCount, maskWords;
    int width, height, rows, rowStart, rowStride;
    int rowBandShift; /* log2 of the rows per band (rtc.h rowBand): 0 = single rows */
    int spp, maxBounce;
    int hoist;
    float invSpp; /* (float)(1. / accumulationCount), main.c:99 */
    V3 origin, ex, ey, ez;
    float fov;
    EnvParams env;
};

/* Data a kernel only reads (written by earlier kernels of the launch) at a wave-uniform address, read through
 * the constant address space so that the compiler issues scalar loads: they return on lgkmcnt,
 * so waiting for one does not also wait for the wave's earlier sample-slot stores to be acknowledged, as a
 * vector load's vmcnt wait does on gfx9 (loads and stores share vmcnt). */
template <typename T> __device__ __forceinline__ const __attribute__((address_space(4))) T *kconst(const T *p)
{
    return (const __attribute__((address_space(4))) T *)p;
}
/* a record of T (a multiple of 4 bytes) from a wave-uniform address, dword by dword through kconst */
template <typename T> __device__ __forceinline__ T kload(const T *p, int i)
{
    static_assert(sizeof(T) % 4 == 0, "dword records");
    T v;
    const __attribute__((address_space(4))) unsigned *q = kconst((const unsigned *)(p + i));
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k)
        ((unsigned *)&v)[k] = q[k];
    return v;
}
#define KCONST(p) kconst(p)
#define KLOAD(p, i) kload(p, i)

/* A RenderParams field of the launch, re-read from the kernarg segment where it is used (KARG; values, and pointers
 * read through KCONST / KLOAD / gload only -- a pointer loaded this way has no known address space, so a plain vector
 * access through it would be a flat one, whose wait covers lgkmcnt too): the kernel's one
 * argument is RenderParams at offset 0 of that segment.  The segment pointer is laundered through an empty asm at every
 * use, so the scalar load is neither hoisted out of the loops nor merged with another use: the field occupies no SGPR
 * between uses.  rtc_render_chain keeps ~60 SGPRs of launch constants (camera, environment, dimensions, pointers)
 * otherwise, and spilled 155 SGPRs to VGPR lanes (v_writelane / v_readlane in its loops).  For fields
 * read once per item, window or escaped bounce: a scalar-cache hit against a register that would have been spilled. */
/* 0 in a vector register the compiler cannot see through: a wave-uniform address plus vzero() is read by a vector load
 * (waited for by vmcnt, in order) instead of a scalar load */
__device__ __forceinline__ int vzero()
{
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
/* a dword of global memory by a global (not flat) vector load: a flat load's wait would also cover the LDS and scalar
 * loads (lgkmcnt) */
template <typename T> __device__ __forceinline__ unsigned gload(const T *p, size_t i)
{
    static_assert(sizeof(T) == 4, "dwords");
    return ((const __attribute__((address_space(1))) unsigned *)p)[i];
}
template <typename T> __device__ __forceinline__ T karg_at(size_t off)
{
    const __attribute__((address_space(4))) char *base =
        (const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(base));
    static_assert(sizeof(T) % 4 == 0, "dword fields");
    T v;
    const __attribute__((address_space(4))) unsigned *q = (const __attribute__((address_space(4))) unsigned *)(base + off);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k)
        ((unsigned *)&v)[k] = q[k];
    return v;
}
/* Contract: KARG(field) names `P`, which must be the calling kernel's one RenderParams argument -- every
 * kernel that uses KARG, directly or through a helper, is declared `kernel(RenderParams P, ...)` with P first, at
 * kernarg offset 0 (rtc_tile_cull, rtc_render_chain), and a helper that uses it takes `const RenderParams &P`.
 * karg_field refuses any other `P` at compile time. */
template <typename PT, typename T> __device__ __forceinline__ T karg_field(size_t off)
{
    static_assert(std::is_same<typename std::decay<PT>::type, RenderParams>::value,
                  "KARG reads the kernel's RenderParams argument: P must be it");
    return karg_at<T>(off);
}
#define KARG(field) karg_field<decltype(P), decltype(RenderParams::field)>(offsetof(RenderParams, field))

constexpr int kTileW = 16, kTileH = 16, kBlock = 256;


/* The pixel a lane renders and its primary ray (rowThread, main.c:88-94).  A 256-thread workgroup covers
 * 16x16 pixels of the launch's rows; wave w of it the 8x8 tile (w & 1, w >> 1). */
struct PixelRay {
    int x, r, y;
    bool valid;
    V3 dir;
};

__device__ __forceinline__ V3 primary_dir(const RenderParams &P, int x, int y)
{
    /* integer halves, then int->float, f32 divide */
    const float dx = (float)(x - P.width / 2) / (float)(P.height / 2);
    const float dy = (float)(y - P.height / 2) / (float)(P.height / 2);
    return normalized(add(add(mul(P.ex, dx), mul(P.ey, dy)), mul(P.ez, P.fov)));
}

/* Launch row r -> image row y: y = rowStart + k*rowStride (main.c:84's interleave), or bands of 2^rowBandShift rows
 * (rtc.h rowBand): y = rowStart + (r / B)*rowStride*B + r % B */
__device__ __forceinline__ int launch_row_y(const RenderParams &P, int r)
{
    const int sh = P.rowBandShift;
    return P.rowStart + ((r >> sh) * P.rowStride << sh) + (r & ((1 << sh) - 1));
}

__device__ __forceinline__ PixelRay pixel_ray(const RenderParams &P, int bx, int by)
{
    PixelRay px;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    px.x = bx * kTileW + (wave & 1) * 8 + (lane & 7);
    px.r = by * kTileH + (wave >> 1) * 8 + (lane >> 3);
    px.valid = px.x < P.width && px.r < P.rows;
    px.y = launch_row_y(P, px.r);
    px.dir = primary_dir(P, px.x, px.y);
    return px;
}

/* This wave's 8x8 tile in the launch (made provably wave-uniform, so tile data is scalar-loaded). */
__device__ __forceinline__ int wave_tile(int bx, int by)
{
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return (by * 2 + (wave >> 1)) * (gridDim.x * 2) + bx * 2 + (wave & 1);
}

/* The workgroup this launch slot renders.  Workgroups are dispatched in launch-slot order; with P.order
 * (rtc_order_blocks) the ones whose pixels see geometry -- the long-running ones -- go first, so the many
 * short sky-only workgroups fill in behind them instead of leaving them as a tail. */
__device__ __forceinline__ void block_xy(const RenderParams &P, int &bx, int &by)
{
    if (P.order) {
        const int id = P.order[blockIdx.y * gridDim.x + blockIdx.x];
        bx = id % (int)gridDim.x;
        by = id / (int)gridDim.x;
    } else {
        bx = blockIdx.x;
        by = blockIdx.y;
    }
}

/* Error bounds for the primary filter (u = 2^-24, |d_i| <= 1 + 2^-22 for a normalized float direction).
 * Reference det: h = cross(d, AC) then a 3-term dot -> |det_e - d.(AC x AB)| <= 5.001 u |AB|_1 |AC|_1.
 * Filter det: FMA dot with Gd rounded to float -> <= 4.004 u |AB|_1 |AC|_1.  Same with s0 for uu; vv uses q0
 * (exact) on both sides (<= 6.002 u |q0|_1); nd uses N on both sides (<= 6.002 u |N|_1).  For u+v > 1 the
 * filter forms w~ = (det~ - u~) - v~ (two more roundings, <= 2.0001 u (|det~| + |u~| + |v~|)) and the
 * reference rejects once sigma*(det - uu - vv) < -2^-21 |det| (three roundings), so that edge carries the
 * three bounds above, the subtraction error and 2^-21 |AB|_1 |AC|_1 (>= |det|).  Every bound is taken 4x and rounded up; the sign tests also carry 2^-60
 * so a product that could round to -0 is never treated as negative. */
__global__ __launch_bounds__(64) void rtc_prep_primary(const DevTri *__restrict__ tris, DevPrimF *__restrict__ pf,
                                                        DevPrimX *__restrict__ px, int triCount, V3 origin,
                                                        int *__restrict__ geoCount)
{
    const int t = blockIdx.x * 64 + threadIdx.x;
    if (geoCount && blockIdx.x == 0 && threadIdx.x < kGeoLists) /* the launch's geometry sub-lists start empty */
        geoCount[threadIdx.x * kGeoCountStride] = 0;
    if (t >= triCount)
        return;
    const DevTri T = tris[t];
    const V3 AB{T.abx, T.aby, T.abz}, AC{T.acx, T.acy, T.acz}, N{T.nx, T.ny, T.nz};
    const V3 s0 = sub(origin, V3{T.ax, T.ay, T.az}); /* raytracing.c:198 */
    const V3 q0 = cross(s0, AB);                      /* :202 */
    const float dac0 = dot(AC, q0);                   /* :206 numerator */
    DevPrimX x;
    x.abx = AB.x, x.aby = AB.y, x.abz = AB.z;
    x.acx = AC.x, x.acy = AC.y, x.acz = AC.z;
    x.s0x = s0.x, x.s0y = s0.y, x.s0z = s0.z;
    x.q0x = q0.x, x.q0y = q0.y, x.q0z = q0.z;
    x.dac0 = dac0;
    x.pad[0] = x.pad[1] = x.pad[2] = 0.f;
    px[t] = x;

    /* exact-math direction vectors, in double, then rounded to float */
    const double abx = AB.x, aby = AB.y, abz = AB.z, acx = AC.x, acy = AC.y, acz = AC.z;
    const double sx = s0.x, sy = s0.y, sz = s0.z;
    const double gdx = acy * abz - acz * aby, gdy = acz * abx - acx * abz, gdz = acx * aby - acy * abx;
    const double gux = acy * sz - acz * sy, guy = acz * sx - acx * sz, guz = acx * sy - acy * sx;
    auto n1 = [](double a, double b, double c) { return fabs(a) + fabs(b) + fabs(c); };
    const double u = 5.9604644775390625e-08; /* 2^-24 */
    const double nAB = n1(abx, aby, abz), nAC = n1(acx, acy, acz), nS = n1(sx, sy, sz);
    const double nQ = n1(q0.x, q0.y, q0.z), nN = n1(N.x, N.y, N.z);
    const double eD = 9.006 * u * nAB * nAC;
    const double eU = 9.006 * u * nS * nAC;
    const double eV = 6.002 * u * nQ;
    const double eW = eD + eU + eV + 2.0002 * u * (nAB * nAC + nS * nAC + nQ) + 4.8e-7 * nAB * nAC;
    const double tiny = 8.673617379884035e-19; /* 2^-60 */
    const double m = fmax(fmax(eU, eV), eW) * 4.0 + tiny;
    const double ed = eD * 4.0;
    const double mnd = 6.002 * u * nN * 4.0;
    /* gigantic or non-finite geometry: disable the filter for this triangle (zero vectors and infinite
     * margins: every finite direction is a candidate and the exact path decides) */
    const bool sane = ed < 2.5e-4 && nAB * nAC < 1e30 && nS * nAC < 1e30 && nQ < 1e30 && m < 1e30 && mnd < 1e30;
    /* dAC0 == 0 (or NaN): dst is 0 or NaN for every ray, which the reference never records */
    const bool never = !(dac0 < 0.f || dac0 > 0.f);
    const float sg = dac0 < 0.f ? -1.f : 1.f;
    DevPrimF f;
    f.nx = N.x, f.ny = N.y, f.nz = N.z;
    f.gdx = sane ? sg * (float)gdx : 0.f, f.gdy = sane ? sg * (float)gdy : 0.f, f.gdz = sane ? sg * (float)gdz : 0.f;
    f.gux = sane ? sg * (float)gux : 0.f, f.guy = sane ? sg * (float)guy : 0.f, f.guz = sane ? sg * (float)guz : 0.f;
    f.q0x = sane ? sg * q0.x : 0.f, f.q0y = sane ? sg * q0.y : 0.f, f.q0z = sane ? sg * q0.z : 0.f;
    f.pad0 = 0.f;
    /* margins rounded outwards to float: sigma*det >= 0.001f (float EPSILON compare, raytracing.c:195) and
     * |det~ - det| <= ed give sigma*det~ >= 0.001f - ed >= c */
    f.mnd = never ? -__builtin_inff() : (sane ? __double2float_ru(mnd) : __builtin_inff());
    f.c = sane ? __double2float_rd((double)0.001f - ed) : -__builtin_inff();
    f.negm = sane ? -__double2float_ru(m) : -__builtin_inff();
    pf[t] = f;
}

struct Closest {
    float dst;
    int idx; /* -1 none; 0..S-1 sphere; S.. triangle (S + t) */
};

/* Exact-safe rejection filter.  With r = rcp(det) (<= 1 ulp) the approximations ua = uu*r, va = vv*r,
 * da = dd*r are within 2^-21 relative of the reference's u, v, dst (raytracing.c:197-207, invDet = 1/det
 * rounded), so each failed comparison below implies the corresponding reference rejection:
 *   ua < -2^-60 => u < 0;  va < -2^-60 => v < 0;  ua+va > 1+1e-5 (ua, va >= -2^-60) => u+v > 1 or u > 1;
 *   da < 0.00099 => dst < EPSILON.
 * The 2^-60 floor keeps the sign tests away from products that could round to -0 (no rejection in the
 * reference).  Every comparison is written so that NaN keeps the lane a candidate: the exact path then
 * decides as the reference does. */
constexpr float kTiny = 8.67361738e-19f; /* 2^-60 */




/* Primary segments (every live lane at bounce 0, pos == camera origin).
 * Filter (per lane, 13 VALU for a front-facing record, 4 for a back-facing one): FMA dot products of the
 * direction with the orientation-folded DevPrimF vectors (sigma = sign(dAC0), see DevPrimF); reject when the
 * bounds prove the reference rejects:
 *   nd > mnd                        => dot(dir, N) > 0                          (raytracing.c:189)
 *   sigma*det~ < c = EPSILON - ed   => |det| < EPSILON or sign(det) != sigma (then dst < 0)   (:195, :206)
 *   min(sigma*u~, sigma*v~, sigma*w~) < -m => u < 0, v < 0 or u+v > 1       (:200-204)
 * The exact reference arithmetic runs only for lanes the filter keeps (NaN directions are never kept:
 * their det is NaN, so the reference cannot record a hit either).  Records are scalar-loaded in batches.
 * prim_backfacing / prim_pass are THE filter: the render kernel and rtc_tile_cull both use them. */
__device__ __forceinline__ float fdot(V3 d, float x, float y, float z) { return fmaf(d.z, z, fmaf(d.y, y, d.x * x)); }

__device__ __forceinline__ bool prim_backfacing(V3 dir, const DevPrimF &F)
{
    return fdot(dir, F.nx, F.ny, F.nz) > F.mnd;
}

__device__ __forceinline__ bool prim_pass(V3 dir, const DevPrimF &F)
{
    const float dt = fdot(dir, F.gdx, F.gdy, F.gdz);
    const float ut = fdot(dir, F.gux, F.guy, F.guz);
    const float vt = fdot(dir, F.q0x, F.q0y, F.q0z);
    const float wt = (dt - ut) - vt;
    return (dt >= F.c) & (fminf(fminf(ut, vt), wt) >= F.negm);
}

/* One primary record (see closest_primary). */
__device__ __forceinline__ void primary_test(const RenderParams &P, V3 dir, const DevPrimF &F, int t, int base,
                                             Closest &c)
{
    if (!prim_backfacing(dir, F)) {
        if (prim_pass(dir, F)) {
            /* the reference's arithmetic (raytracing.c:189-208) */
            const DevPrimX X = P.primX[t];
            if (!(dot(dir, V3{F.nx, F.ny, F.nz}) >= 0.f)) {
                const V3 h = cross(dir, V3{X.acx, X.acy, X.acz});
                const float det = dot(V3{X.abx, X.aby, X.abz}, h);
                if (!(-kEps < det && det < kEps)) {
                    const float invDet = rcp_cr(det); /* IEEE 1.f / det */
                    const float u = dot(V3{X.s0x, X.s0y, X.s0z}, h) * invDet;
                    const float v = dot(dir, V3{X.q0x, X.q0y, X.q0z}) * invDet;
                    const float dst = X.dac0 * invDet;
                    if (!(u < 0.f || u > 1.f) && !(v < 0.f || u + v > 1.f) && !(dst < kEps) && dst < c.dst) {
                        c.dst = dst;
                        c.idx = base + t;
                    }
                }
            }
        }
    }
}

/* Brute force over every record (RTC_F_NO_TILE_CULL).  Records are scalar-loaded in two alternating
 * batches of kUnroll: the next batch is in flight while the current one is tested (the arrays carry 8 spare
 * records so the last prefetch stays in bounds). */
__device__ __forceinline__ void closest_primary(const RenderParams &P, V3 dir, Closest &c, int base)
{
    const DevPrimF *rec = P.primF;
    DevPrimF A[kUnroll], B[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k)
        A[k] = rec[k];
    for (int t0 = 0; t0 < P.triPadded; t0 += 2 * kUnroll, rec += 2 * kUnroll) {
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            B[k] = rec[kUnroll + k];
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            primary_test(P, dir, A[k], t0 + k, base, c);
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            A[k] = rec[2 * kUnroll + k];
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            primary_test(P, dir, B[k], t0 + kUnroll + k, base, c);
    }
}

/* Only the tile's candidates (rtc_tile_cull), in ascending index order, so ties keep the lowest index as
 * calculateRayCollision's strict `<` does (raytracing.c:231).  `mask` is wave-uniform: the bit-set words
 * and the records are scalar loads. */
__device__ __forceinline__ void closest_primary_listed(const RenderParams &P, V3 dir, Closest &c, int base,
                                                       const unsigned long long *__restrict__ mask)
{
    for (int w = 0; w < P.maskWords; ++w) {
        unsigned long long m = mask[w];
        while (m) {
            const int t = w * 64 + __builtin_ctzll(m);
            m &= m - 1;
            primary_test(P, dir, P.primF[t], t, base, c);
        }
    }
}

/* General segments (any origin): rayTriangle (raytracing.c:186-214) with AB, AC precomputed.
 * general_filter: the exact-safe rejection (backface, |det| < EPSILON, u out of range by the rcp estimate);
 * general_exact: the reference's arithmetic for a record the filter keeps (recomputes the same values). */
__device__ __forceinline__ bool general_filter(V3 pos, V3 dir, const DevTri &R)
{
    const float nd = dot(dir, V3{R.nx, R.ny, R.nz});
    const V3 AB{R.abx, R.aby, R.abz}, AC{R.acx, R.acy, R.acz};
    const V3 h = cross(dir, AC);
    const float det = dot(AB, h);
    const V3 s = sub(pos, V3{R.ax, R.ay, R.az});
    const float uu = dot(s, h);
    const float ua = uu * __builtin_amdgcn_rcpf(det);
    const bool detOk = !(-kEps < det && det < kEps);
    return (int)!(nd >= 0.f) & (int)detOk & (int)!(ua < -kTiny) & (int)!(ua > 1.000001f);
}

__device__ __forceinline__ void general_exact(V3 pos, V3 dir, const DevTri &R, int idx, Closest &c)
{
    const V3 AB{R.abx, R.aby, R.abz}, AC{R.acx, R.acy, R.acz};
    const V3 h = cross(dir, AC);
    const float det = dot(AB, h);
    const V3 s = sub(pos, V3{R.ax, R.ay, R.az});
    const float invDet = rcp_cr(det); /* IEEE 1.f / det */
    const float u = dot(s, h) * invDet;
    const V3 q = cross(s, AB);
    const float v = dot(dir, q) * invDet;
    const float dst = dot(AC, q) * invDet;
    /* records may be visited out of index order (clusters): equal distances keep the lowest index, as the
     * reference's strict `<` over ascending indices does (raytracing.c:231) */
    if (!(u < 0.f || u > 1.f) && !(v < 0.f || u + v > 1.f) && !(dst < kEps) &&
        (dst < c.dst || (dst == c.dst && (unsigned)idx < (unsigned)c.idx))) {
        c.dst = dst;
        c.idx = idx;
    }
}

__device__ __forceinline__ void general_test(V3 pos, V3 dir, const DevTri &R, int idx, Closest &c)
{
    const float nd = dot(dir, V3{R.nx, R.ny, R.nz});
    if (!(nd >= 0.f)) {
        const V3 AB{R.abx, R.aby, R.abz}, AC{R.acx, R.acy, R.acz};
        const V3 h = cross(dir, AC);
        const float det = dot(AB, h);
        const V3 s = sub(pos, V3{R.ax, R.ay, R.az});
        const float uu = dot(s, h);
        const float r = __builtin_amdgcn_rcpf(det);
        const float ua = uu * r;
        const bool detOk = !(-kEps < det && det < kEps);
        if (detOk & !(ua < -kTiny) & !(ua > 1.000001f)) {
            const float invDet = rcp_cr(det); /* IEEE 1.f / det */
            const float u = uu * invDet;
            const V3 q = cross(s, AB);
            const float v = dot(dir, q) * invDet;
            const float dst = dot(AC, q) * invDet;
            if (!(u < 0.f || u > 1.f) && !(v < 0.f || u + v > 1.f) && !(dst < kEps) && dst < c.dst) {
                c.dst = dst;
                c.idx = idx;
            }
        }
    }
}

/* Scenes up to kLdsTris triangles keep their general-path records in LDS (one copy per workgroup, loaded at
 * kernel start): the general loop then reads them as broadcast ds_read_b128 instead of scalar loads that
 * compete for the scalar cache with the primary records. */
constexpr int kLdsTris = 256;

__device__ __forceinline__ void closest_general_lds(const DevTri *__restrict__ lds, int Tp, V3 pos, V3 dir,
                                                    Closest &c, int base)
{
    for (int t0 = 0; t0 < Tp; t0 += 2) {
        const DevTri R0 = lds[t0], R1 = lds[t0 + 1];
        general_test(pos, dir, R0, base + t0, c);
        general_test(pos, dir, R1, base + t0 + 1, c);
    }
}

__device__ __forceinline__ void closest_general(const RenderParams &P, V3 pos, V3 dir, Closest &c, int base)
{
    const int Tp = P.triPadded;
    /* two alternating scalar-load batches, as closest_primary: the next records are in flight while the
     * current ones are tested (the arrays carry 8 spare records) */
    const DevTri *rec = P.tris;
    DevTri A[kUnroll], B[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k)
        A[k] = rec[k];
    for (int t0 = 0; t0 < Tp; t0 += 2 * kUnroll, rec += 2 * kUnroll) {
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            B[k] = rec[kUnroll + k];
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            general_test(pos, dir, A[k], base + t0 + k, c);
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            A[k] = rec[2 * kUnroll + k];
#pragma unroll
        for (int k = 0; k < kUnroll; ++k)
            general_test(pos, dir, B[k], base + t0 + kUnroll + k, c);
    }
}

/* calculateRayCollision (raytracing.c:216-240): spheres first (only if !trianglesOnly), then triangles
 * in index order; a candidate replaces the current one only if strictly closer (ties keep the lower
 * index).  The loop trip counts are kernel arguments, so the triangle index is wave-uniform and its
 * record is fetched with scalar loads.  `primaryWave` (wave-uniform) = every live lane is at bounce 0;
 * `mask` (wave-uniform, nullable) = the tile's primary candidates. */
template <bool SPHERES>
__device__ __forceinline__ Closest closest_hit(const RenderParams &P, V3 pos, V3 dir, bool primaryWave,
                                               const unsigned long long *mask, const DevTri *lds)
{
    Closest c{999999.f, -1};
    if (SPHERES) {
        for (int i = 0; i < P.sphereCount; ++i) {
            const DevSphere sp = P.spheres[i];
            float d;
            if (ray_sphere(pos, dir, V3{sp.cx, sp.cy, sp.cz}, sp.radius, d) && d < c.dst) {
                c.dst = d;
                c.idx = i;
            }
        }
    }
    const int base = SPHERES ? P.sphereCount : 0;
    if (primaryWave) {
        if (mask)
            closest_primary_listed(P, dir, c, base, mask);
        else
            closest_primary(P, dir, c, base);
    } else if (lds) {
        closest_general_lds(lds, P.triPadded, pos, dir, c, base);
    } else {
        closest_general(P, pos, dir, c, base);
    }
    return c;
}

#ifdef RTC_DIAG
/* diagnostic build only (librtc_diag.so): per-wave {cycles, wave-loop iterations, start stamp, cycles inside
 * closest_hit} */
__device__ unsigned long long *g_rtc_diag = nullptr;
extern "C" int rtc_diag_set_buffer(void *dptr)
{
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rtc_diag), &dptr, sizeof dptr));
    return 0;
}
/* heavy-kernel section cycles (s_memtime deltas summed over waves): 0 primary trace, 1 cluster tests,
 * 2 general filter loop, 3 general exact loop, 4 lane reduction, 5 hit shading, 6 sky (miss), 7 loop total */
constexpr int kDiagSects = 24;
__device__ unsigned long long g_rtc_sect[kDiagSects]; /* [8..12] window statistics (rtc_render_chain) */
/* rtc_render_chain's diagnostics, written with plain stores to per-wave-slot / per-item addresses (no same-address global
 * atomics: thousands of them queued at a kernel's end held up other waves' memory operations behind them in the L2
 * channels and made the tail look slow):
 *   g_rtc_wavelog[slot]: start, end, items, the end of items 1..5 (s_memrealtime, the 100 MHz constant clock);
 *   g_rtc_sectw[slot]: the wave's section cycles (s_rtc_sect) and window statistics, summed by rtc_diag_sections;
 *   g_rtc_itemlog[item]: (start, end), (windows | tile candidates << 16 | wave slot << 32), (bounce iterations |
 *     Box-Muller fallback lanes << 16 | triangle tests of the window lanes << 32, RTC_DIAG_COUNT builds only);
 *   g_rtc_itemsect[item]: the item's cycles in sections kItemSectIds (s_memtime deltas). */
constexpr int kWaveLog = 16384, kWaveLogCols = 8;
__device__ unsigned long long g_rtc_wavelog[kWaveLog][kWaveLogCols];
__device__ unsigned long long g_rtc_sectw[kWaveLog][kDiagSects];
constexpr int kItemLog = 1 << 18, kItemSectLog = 1 << 17, kItemSects = 16;
__device__ unsigned long long g_rtc_itemlog[kItemLog][4];
__device__ unsigned g_rtc_itemsect[kItemSectLog][kItemSects];
__device__ __forceinline__ int item_sect_id(int k) /* the sections of g_rtc_itemsect's columns */
{
    return k < 10 ? k : (k == 10 ? 14 : k + 4); /* columns 0..9: sections 0..9; 10: 14; 11..15: 15..19 */
}
template <typename T> static int diag_zero(const T &sym)
{
    void *p = nullptr;
    HIP_TRY(hipGetSymbolAddress(&p, HIP_SYMBOL(sym)));
    HIP_TRY(hipMemset(p, 0, sizeof(T)));
    return 0;
}
extern "C" int rtc_diag_itemlog(unsigned long long *out, int maxItems)
{
    const int n = std::min(maxItems, kItemLog);
    if (out && n > 0)
        HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtc_itemlog), (size_t)n * 4 * sizeof(unsigned long long)));
    return n;
}
extern "C" int rtc_diag_itemsect(unsigned *out, int maxItems)
{
    const int n = std::min(maxItems, kItemSectLog);
    if (out && n > 0)
        HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtc_itemsect), (size_t)n * kItemSects * sizeof(unsigned)));
    return n;
}
/* the wave records of the last launches (rows with a zero start: no wave); returns the slots copied */
extern "C" int rtc_diag_wavelog(unsigned long long *out, int maxWaves, int reset)
{
    const int n = std::min(maxWaves, kWaveLog);
    if (out && n > 0)
        HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtc_wavelog), (size_t)n * kWaveLogCols * sizeof(unsigned long long)));
    if (reset && diag_zero(g_rtc_wavelog))
        return -1;
    return n;
}
#define CSTAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
/* per-block records of rtc_tile_cull (wave 0): {start, level 1 done, end, geometry, level-2 prefilter cycles, candidate
 * loop cycles, candidates, 0}, written with plain stores into the buffer rtc_diag_set_cull_buffer names (null: none) */
__device__ unsigned long long *g_rtc_cullwg = nullptr;
extern "C" int rtc_diag_set_cull_buffer(void *dptr)
{
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rtc_cullwg), &dptr, sizeof dptr));
    return 0;
}
#define CREC(blk, a, b, c, geo, pre, loop, cand)                                                              \
    do {                                                                                                       \
        if (g_rtc_cullwg && threadIdx.x == 0) {                                                                \
            unsigned long long *r_ = g_rtc_cullwg + (size_t)(blk) * 8;                                         \
            r_[0] = (a), r_[1] = (b), r_[2] = (c), r_[3] = (geo), r_[4] = (pre), r_[5] = (loop), r_[6] = (cand); \
        }                                                                                                      \
    } while (0)
__shared__ unsigned long long s_rtc_sect[4][kDiagSects]; /* [wave][section]: 0..7, 13..23 (rtc_render_chain) */
#define DSECT_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define DSECT_END(v, k)                                                                                        \
    do {                                                                                                       \
        const unsigned long long dsectNow = __builtin_amdgcn_s_memtime();                                      \
        if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63))                           \
            s_rtc_sect[threadIdx.x >> 6][k] += dsectNow - (v);                                                 \
    } while (0)
/* Uniform section marks: the cycles since the previous mark of the wave go to section k.  Placed at wave-uniform points
 * only, the marks tile the loop: every cycle between the kernel's first mark and its last lands in exactly one section
 * (the BEGIN/END pairs above nest inside them) */
#define DMARK_INIT(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define DMARK(v, k)                                                                                            \
    do {                                                                                                       \
        const unsigned long long dmarkNow = __builtin_amdgcn_s_memtime();                                      \
        if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63))                           \
            s_rtc_sect[threadIdx.x >> 6][k] += dmarkNow - (v);                                                 \
        (v) = dmarkNow;                                                                                        \
    } while (0)
extern "C" int rtc_diag_sections(unsigned long long *out, int reset)
{
    /* out: kDiagSects (24) counters */
    if (out) {
        HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rtc_sect), kDiagSects * sizeof(unsigned long long)));
        std::vector<unsigned long long> w((size_t)kWaveLog * kDiagSects);
        HIP_TRY(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_rtc_sectw), w.size() * sizeof(unsigned long long)));
        for (size_t i = 0; i < w.size(); ++i)
            out[i % kDiagSects] += w[i];
    }
    if (reset) {
        unsigned long long z[kDiagSects] = {0};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rtc_sect), z, sizeof z));
        if (diag_zero(g_rtc_sectw))
            return -1;
    }
    return 0;
}
#else
#define DSECT_BEGIN(v) (void)0
#define DSECT_END(v, k) (void)0
#define DMARK_INIT(v) (void)0
#define DMARK(v, k) (void)0
#define CSTAMP(v) (void)0
#define CREC(blk, a, b, c, geo, pre, loop, cand) (void)0
#endif

/* Tile candidate lists for primary segments.  A pixel's primary ray is the same ray for every sample
 * (main.c:88-94: no jitter), so the primary filter's verdict for (pixel, triangle) is the same for
 * every sample.  One pass over the launch's pixels records, per 8x8 tile (= one wave of the render kernel),
 * the set of triangles the filter keeps for at least one pixel of the tile; the render kernel's primary
 * segments then visit only that set, in index order.  A triangle left out fails the filter for every pixel
 * of the tile, so the reference's rayTriangle rejects it for every primary ray there: the closest hit is
 * unchanged, bit for bit.  The filter is the render kernel's own (prim_backfacing / prim_pass, same records,
 * same pixel_ray). */
/* Tile prefilter.  The per-pixel filter values nd, dt, ut, vt, wt are (FMA) dot products of the pixel's f32
 * direction d with per-triangle vectors g.  Over an 8x8 tile, d = v / |v| with v = ex dx + ey dy + ez fov
 * affine in the pixel's (dx, dy), which lie in the rectangle spanned by the tile's extreme pixels (dx, dy
 * are monotone in x, y).  So g.v takes its extremes at the rectangle's corners, |v| lies in [vmin, vmax]
 * (vmax: |v| is convex, a corner; vmin: v.ez/|ez| is affine, its smallest corner value, when positive), and
 * g.d (exact direction) lies in [LB, UB] with UB = Amax / vmin or Amax / vmax by the sign of the corner
 * maximum Amax (LB likewise).  The computed value differs from g.d(exact) by at most
 *   |g|_1 (eDir + 3.01 u),  eDir = 16 u S / vmin + 4 u  (u = 2^-24, S = max|dx| + max|dy| + |fov|)
 * (f32 v: 3 roundings per component, <= 3 u S each; normalisation <= 2 u; the FMA dot <= 3 u |g|_1; the
 * constants carry ~1.5x).  A triangle is left out of the tile when one filter condition fails for every
 * point of that range -- then it fails for every pixel, exactly as the per-pixel filter would decide.
 * Computed in double per (tile, triangle); a tile whose bounds are not finite or whose vmin <= 0 is never
 * pruned. */
struct TileCone {
    double c[4][3];
    double vmin, vmax, eDir;
    double ivmin, ivmax; /* 1 / vmin, 1 / vmax (cone_range multiplies and widens instead of dividing) */
    bool ok;
};

/* the cone of the pixel rectangle [x0, x1] x [r0, r1] (launch rows) */
__device__ TileCone rect_cone(const RenderParams &P, int x0, int x1, int r0, int r1)
{
    TileCone K;
    x1 = min(x1, P.width - 1);
    r1 = min(r1, P.rows - 1);
    const int y0 = launch_row_y(P, r0), y1 = launch_row_y(P, r1); /* (y is increasing in the launch row) */
    /* the same f32 expressions as primary_dir */
    const float dxs[2] = {(float)(x0 - P.width / 2) / (float)(P.height / 2),
                          (float)(x1 - P.width / 2) / (float)(P.height / 2)};
    const float dys[2] = {(float)(y0 - P.height / 2) / (float)(P.height / 2),
                          (float)(y1 - P.height / 2) / (float)(P.height / 2)};
    const double ezl = sqrt((double)P.ez.x * P.ez.x + (double)P.ez.y * P.ez.y + (double)P.ez.z * P.ez.z);
    double vmin = 1e300, vmax = 0.0;
    bool finite = ezl > 0.0 && ezl < 1e300;
    for (int k = 0; k < 4; ++k) {
        const double dx = dxs[k & 1], dy = dys[k >> 1];
        const double v[3] = {(double)P.ex.x * dx + (double)P.ey.x * dy + (double)P.ez.x * P.fov,
                             (double)P.ex.y * dx + (double)P.ey.y * dy + (double)P.ez.y * P.fov,
                             (double)P.ex.z * dx + (double)P.ey.z * dy + (double)P.ez.z * P.fov};
        for (int i = 0; i < 3; ++i) {
            K.c[k][i] = v[i];
            finite = finite && (v[i] - v[i] == 0.0);
        }
        vmax = fmax(vmax, sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]));
        vmin = fmin(vmin, (v[0] * P.ez.x + v[1] * P.ez.y + v[2] * P.ez.z) / ezl);
    }
    const double u = 5.9604644775390625e-08;
    const double S = fmax(fabs((double)dxs[0]), fabs((double)dxs[1])) + fmax(fabs((double)dys[0]), fabs((double)dys[1])) +
                     fabs((double)P.fov);
    K.vmin = vmin * (1.0 - 1e-12);
    K.vmax = vmax * (1.0 + 1e-12);
    K.eDir = 16.0 * u * S / K.vmin + 4.0 * u;
    K.ivmin = 1.0 / K.vmin;
    K.ivmax = 1.0 / K.vmax;
    /* basis components <= 1 (normalized f32 vectors) is assumed by the error bound */
    const bool unitBasis = fabs(P.ex.x) <= 1.0001f && fabs(P.ex.y) <= 1.0001f && fabs(P.ex.z) <= 1.0001f &&
                           fabs(P.ey.x) <= 1.0001f && fabs(P.ey.y) <= 1.0001f && fabs(P.ey.z) <= 1.0001f &&
                           fabs(P.ez.x) <= 1.0001f && fabs(P.ez.y) <= 1.0001f && fabs(P.ez.z) <= 1.0001f;
    K.ok = finite && unitBasis && K.vmin > 1e-6 && K.eDir < 1e-3 && S - S == 0.0;
    return K;
}

__device__ TileCone tile_cone(const RenderParams &P, int tx, int ty)
{
    return rect_cone(P, tx * 8, tx * 8 + 7, ty * 8, ty * 8 + 7);
}

/* [LB, UB] of g.v/|v| over the tile (see TileCone) */
__device__ __forceinline__ void cone_range(const TileCone &K, double gx, double gy, double gz, double &lb, double &ub)
{
    double mx = -1e300, mn = 1e300;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double a = gx * K.c[k][0] + gy * K.c[k][1] + gz * K.c[k][2];
        mx = fmax(mx, a);
        mn = fmin(mn, a);
    }
    /* mx / vmin (or / vmax) as a product with the rounded reciprocal: two double roundings, < 2^-51 relative, so
     * widening by 2^-50 of the magnitude keeps ub above (lb below) the exact quotient -- the bound only loosens */
    ub = mx * (mx >= 0.0 ? K.ivmin : K.ivmax);
    lb = mn * (mn >= 0.0 ? K.ivmax : K.ivmin);
    ub += fabs(ub) * 0x1p-50;
    lb -= fabs(lb) * 0x1p-50;
}

/* true: no pixel of the tile can pass prim_backfacing / prim_pass for F */
__device__ bool tile_prunes(const TileCone &K, const DevPrimF &F)
{
    const double u = 5.9604644775390625e-08;
    const double e = K.eDir + 3.01 * u;
    auto n1 = [](double a, double b, double c) { return fabs(a) + fabs(b) + fabs(c); };
    double lb, ub;
    /* every pixel back-facing: nd > mnd */
    cone_range(K, F.nx, F.ny, F.nz, lb, ub);
    if (lb - n1(F.nx, F.ny, F.nz) * e > (double)F.mnd)
        return true;
    const double nd = n1(F.gdx, F.gdy, F.gdz), nu = n1(F.gux, F.guy, F.guz), nv = n1(F.q0x, F.q0y, F.q0z);
    cone_range(K, F.gdx, F.gdy, F.gdz, lb, ub);
    if (ub + nd * e < (double)F.c)
        return true;
    cone_range(K, F.gux, F.guy, F.guz, lb, ub);
    if (ub + nu * e < (double)F.negm)
        return true;
    cone_range(K, F.q0x, F.q0y, F.q0z, lb, ub);
    if (ub + nv * e < (double)F.negm)
        return true;
    /* wt = (dt - ut) - vt: the three slacks plus two f32 subtractions */
    cone_range(K, (double)F.gdx - F.gux - F.q0x, (double)F.gdy - F.guy - F.q0y, (double)F.gdz - F.guz - F.q0z, lb,
               ub);
    if (ub + (nd + nu + nv) * (e + 2.01 * u * 1.0001) < (double)F.negm)
        return true;
    return false;
}

/* Level 0 of the tile cull: the same prefilter over a superblock of kSuperBlocks x kSuperBlocks workgroup blocks (64 x 64
 * pixels of the launch's rows), one wave each.  A triangle it prunes fails the filter for every pixel of the superblock,
 * so rtc_tile_cull's level 1 tests only its survivors, and a block whose superblock keeps none (the sky of a frame)
 * skips its own double-precision cone.  Same candidate lists bit for bit (each level only removes triangles the
 * per-pixel filter rejects for every pixel of the rectangle). */
constexpr int kSuperBlocks = 4;
/* (launches of more than rtcplan::kSuperCullPixels pixels run level 0) */
__global__ __launch_bounds__(64) void rtc_super_cull(RenderParams P, unsigned long long *__restrict__ superMask)
{
    const int sx = blockIdx.x, sy = blockIdx.y, lane = threadIdx.x;
    const int x0 = sx * kSuperBlocks * kTileW, r0 = sy * kSuperBlocks * kTileH;
    const TileCone K = rect_cone(P, x0, x0 + kSuperBlocks * kTileW - 1, r0, r0 + kSuperBlocks * kTileH - 1);
    unsigned long long *out = superMask + (size_t)(sy * P.superX + sx) * P.maskWords;
    for (int w = 0; w < P.maskWords; ++w) {
        const int ti = w * 64 + lane;
        const bool maybe = ti < P.triPadded && (!K.ok || !tile_prunes(K, P.primF[ti]));
        const unsigned long long m = __ballot(maybe);
        if (lane == 0)
            out[w] = m;
    }
}

/* Outputs: pixMask (every tile: its pixels with a candidate) and, for the split launch (P.geoList), the candidate words
 * of the workgroups with a surviving triangle and the geometry-pixel lists: rtc_render_chain reads the words of the
 * tiles its items lie in, the sky pass pixMask alone.  Round 6: a split launch no longer writes the zero words of the
 * workgroups without a survivor (most of a sky-heavy frame), a per-tile pixel count or the workgroup weights (only
 * rtc_order_blocks reads those, before the one-lane-per-pixel kernel): WRITE_SIZE per 1080p launch 2.13 -> 0.88 MB, the
 * frame unchanged (profiles/r06_j_pmc_writes.log, r06_i_ab_cull_trim_xcd_runs_prefetch.log). */
__global__ __launch_bounds__(kBlock) void rtc_tile_cull(RenderParams P, unsigned long long *__restrict__ mask,
                                                       unsigned *__restrict__ weight,
                                                       unsigned long long *__restrict__ pixMask)
{
    const bool split = P.geoList != nullptr; /* (uniform) */
    if (KARG(cullPrio)) /* (RenderParams::cullPrio) */
        __builtin_amdgcn_s_setprio(3);
    __shared__ unsigned wgWeight, wgAny;
    extern __shared__ unsigned long long sBlockCand[]; /* maskWords: the block's 16x16 prefilter survivors */
    CSTAMP(c0);
    if (threadIdx.x == 0) {
        wgWeight = 0;
        wgAny = 0;
    }
    const int bx = blockIdx.x, by = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (P.geoCountNext && bx == 0 && by == 0 && threadIdx.x < kGeoLists) /* the next split launch's sub-lists */
        P.geoCountNext[threadIdx.x * kGeoCountStride] = 0;
    /* level 1: the prefilter over the workgroup's 16x16 pixels (a superset of each tile's direction range, so
     * a triangle it prunes fails for every pixel of the four tiles); the waves share the mask words */
    __syncthreads();
    /* the superblock's survivors (level 0, rtc_super_cull; all ones without it): wave-uniform scalar loads */
    const unsigned long long *sup =
        P.superMask ? P.superMask + (size_t)((by / kSuperBlocks) * P.superX + bx / kSuperBlocks) * P.maskWords : nullptr;
    bool supAny = !sup;
    for (int w = 0; sup && w < P.maskWords && !supAny; ++w)
        supAny = KCONST(sup)[w] != 0ull;
    if (wave < P.maskWords && supAny) { /* wave-uniform: only the waves with mask words need the block's cone */
        const TileCone KB = rect_cone(P, bx * kTileW, bx * kTileW + kTileW - 1, by * kTileH, by * kTileH + kTileH - 1);
        for (int w = wave; w < P.maskWords; w += kBlock / 64) {
            const int ti = w * 64 + lane;
            const unsigned long long sw = sup ? KCONST(sup)[w] : ~0ull;
            const bool maybe = ((sw >> lane) & 1ull) && ti < P.triPadded &&
                               (!KB.ok || !tile_prunes(KB, P.primF[ti]));
            const unsigned long long m = __ballot(maybe);
            if (lane == 0) {
                sBlockCand[w] = m;
                if (m)
                    wgAny = 1; /* benign race: every writer stores 1 */
            }
        }
    }
    __syncthreads();
    CSTAMP(c1);
    const int tile = wave_tile(bx, by);
    unsigned long long *out = mask + (size_t)tile * P.maskWords;
    if (!wgAny) { /* workgroup-uniform: no triangle survives for any of its pixels (most of a sky-heavy frame) */
        for (int w = lane; !split && w < P.maskWords; w += 64)
            out[w] = 0ull;
        if (lane == 0)
            pixMask[tile] = 0ull;
        if (threadIdx.x == 0 && !split)
            weight[blockIdx.y * gridDim.x + blockIdx.x] = 0u;
        CSTAMP(c9);
        CREC(blockIdx.y * gridDim.x + blockIdx.x, c0, c1, c9, 0, 0, 0, 0);
        return;
    }
#ifdef RTC_DIAG
    unsigned long long dPre = 0, dLoop = 0, dCand = 0;
#endif
    const PixelRay px = pixel_ray(P, bx, by);
    bool anyCand = false;
    /* level 2: the tile's own prefilter on the block's survivors, then the per-pixel filter */
    const TileCone K = tile_cone(P, tile % (int)(gridDim.x * 2), tile / (int)(gridDim.x * 2));
    for (int w = 0; w < P.maskWords; ++w) {
        /* lane l: may triangle 64w + l pass for some pixel of the tile? */
        const int ti = w * 64 + lane;
        const unsigned long long bc = sBlockCand[w];
        CSTAMP(c2);
        const bool maybe = ((bc >> lane) & 1ull) && (!K.ok || !tile_prunes(K, P.primF[ti]));
        unsigned long long todo = bc ? __ballot(maybe) : 0ull;
        unsigned long long bits = 0;
        CSTAMP(c3);
#ifdef RTC_DIAG
        dPre += c3 - c2;
        dCand += (unsigned long long)__popcll(todo);
#endif
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const DevPrimF F = KLOAD(P.primF, w * 64 + j);
            const bool keep = (int)px.valid & (int)!prim_backfacing(px.dir, F) & (int)prim_pass(px.dir, F);
            anyCand |= keep;
            if (__ballot(keep))
                bits |= 1ull << j;
        }
        CSTAMP(c4);
#ifdef RTC_DIAG
        dLoop += c4 - c3;
#endif
        if (lane == 0)
            out[w] = bits;
    }
    /* the tile's pixels with at least one candidate (they do the bounce work); a tile has a non-empty candidate list
     * exactly when one of them is set */
    const unsigned long long b = __ballot(anyCand);
    if (lane == 0)
        pixMask[tile] = b;
    if (P.geoList && b) {
        /* this tile's geometry pixels, appended to sub-list tile % kGeoLists (rtc_render_chain's work) */
        const auto append = [&](unsigned long long gb, int l) {
            int base = 0;
            if (lane == 0)
                base = atomicAdd(&P.geoCount[l * kGeoCountStride], __popcll(gb));
            base = __builtin_amdgcn_readfirstlane(base);
            /* a sub-list holds every geometry pixel of its tiles (geoCap = 64 x its tiles) when its counter started at
             * 0; a stale counter must not write past it (the readers clamp the counts to geoCap too) */
            if (((gb >> lane) & 1ull) && base + __popcll(gb) <= P.geoCap) {
                const int pos = base + __popcll(gb & ((1ull << lane) - 1ull));
                P.geoList[(size_t)l * P.geoCap + pos] = tile * 64 + lane;
                if (P.pixItem) /* the pixel's entry: pos of sub-list l (the sky pass turns it into its item) */
                    P.pixItem[(size_t)tile * 64 + lane] = (unsigned)(pos * kGeoLists + l);
            }
        };
        append(b, tile % kGeoLists);
    }
    if (!split) { /* the one-lane-per-pixel kernel's workgroup order (rtc_order_blocks) */
        if (lane == 0 && b)
            atomicAdd(&wgWeight, (unsigned)__popcll(b));
        __syncthreads();
        if (threadIdx.x == 0)
            weight[blockIdx.y * gridDim.x + blockIdx.x] = wgWeight;
    }
    CSTAMP(c6);
#ifdef RTC_DIAG
    CREC(blockIdx.y * gridDim.x + blockIdx.x, c0, c1, c6, 1, dPre, dLoop, dCand);
#endif
}

/* Launch order of the render kernel's workgroups: a counting sort of the weights, heaviest bucket first
 * (order inside a bucket is arbitrary; the frame does not depend on it -- every pixel is seeded by its own
 * index, main.c:95).  One workgroup; n is at most a few ten thousand. */
constexpr int kOrderBuckets = 17; /* weight / 16: 0 (sky only) .. 16 (all 256 pixels see geometry) */
__global__ __launch_bounds__(1024) void rtc_order_blocks(const unsigned *__restrict__ weight, int n,
                                                          int *__restrict__ order)
{
    __shared__ int cnt[kOrderBuckets];
    if (threadIdx.x < kOrderBuckets)
        cnt[threadIdx.x] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        atomicAdd(&cnt[min(kOrderBuckets - 1, (int)((weight[i] + 15) / 16))], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int off = 0;
        for (int b = kOrderBuckets - 1; b >= 0; --b) {
            const int c = cnt[b];
            cnt[b] = off;
            off += c;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        order[atomicAdd(&cnt[min(kOrderBuckets - 1, (int)((weight[i] + 15) / 16))], 1)] = i;
}

/* Segment counters.  One atomic per wave into the caller's three counters serialises in L2 (tens of
 * thousands of same-address atomics per frame cost milliseconds), so waves add into kSegSlots slots, each
 * in its own 128-B line, and rtc_reduce_segments folds the slots into the caller's counters at the end. */
constexpr int kSegSlots = 256, kSegSlotStride = 16; /* u64 */
static_assert(kSegSlots * kSegSlotStride == 256 * 16, "rtc_scene_upload allocates 256 x 16 u64");

/* counters (rtc.h RTC_SEGMENT_COUNTERS): [0] calculateRayCollision calls, [1] traced, [2] ray-triangle tests of
 * the accumulated samples, [3] ray-cluster tests, [4] ray-triangle tests of speculative samples that were
 * evaluated but not accumulated (rtc_render_chain window lanes off the chain) */
__device__ __forceinline__ void flush_counters(const RenderParams &P, unsigned segCalls, unsigned segTraced,
                                               unsigned long long segTests, int lane, unsigned segClusters = 0,
                                               unsigned long long segSpec = 0)
{
    if (!P.segments)
        return;
    unsigned long long a = segCalls, b = segTraced, n = segTests, k = segClusters, q = segSpec;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
        n += __shfl_xor(n, off);
        k += __shfl_xor(k, off);
        q += __shfl_xor(q, off);
    }
    if (lane == 0 && (a | b | n | k | q)) {
        const unsigned slot = (blockIdx.x * 7u + blockIdx.y * 131u + (threadIdx.x >> 6)) % kSegSlots;
        unsigned long long *c = P.segSlots + (size_t)slot * kSegSlotStride;
        atomicAdd(&c[0], a);
        atomicAdd(&c[1], b);
        atomicAdd(&c[2], n);
        if (k)
            atomicAdd(&c[3], k);
        if (q)
            atomicAdd(&c[4], q);
    }
}

__global__ __launch_bounds__(kSegSlots) void rtc_reduce_segments(unsigned long long *__restrict__ slots,
                                                                 unsigned long long *__restrict__ out)
{
    __shared__ unsigned long long part[RTC_SEGMENT_COUNTERS][kSegSlots / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int k = 0; k < RTC_SEGMENT_COUNTERS; ++k) {
        unsigned long long v = slots[(size_t)t * kSegSlotStride + k];
        slots[(size_t)t * kSegSlotStride + k] = 0; /* zero again for the next launch */
        for (int off = 32; off > 0; off >>= 1)
            v += __shfl_xor(v, off);
        if (lane == 0)
            part[k][w] = v;
    }
    __syncthreads();
    if (t < RTC_SEGMENT_COUNTERS) {
        unsigned long long v = 0;
        for (int i = 0; i < kSegSlots / 64; ++i)
            v += part[t][i];
        out[t] += v; /* stream-ordered after every render kernel of the launch: no atomic needed */
    }
}


template <bool SPHERES, bool DEBUG>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1))) void rtc_render_kernel(
    RenderParams P)
{
#ifdef RTC_DIAG
    const unsigned long long diagT0 = __builtin_amdgcn_s_memtime();
    unsigned diagIters = 0;
    unsigned long long diagTrace = 0;
#endif
    const int lane = threadIdx.x & 63;
    int bx, by;
    block_xy(P, bx, by);
    const PixelRay px = pixel_ray(P, bx, by);
    const int x = px.x, r = px.r, y = px.y;
    const bool valid = px.valid;
    const V3 pdir = px.dir;
    unsigned rng = (unsigned)(x + y * P.width); /* main.c:95 */

    /* general-path records in LDS (small scenes) and the powf tables */
    __shared__ DevTri sTris[kLdsTris];
    __shared__ PowTablesLds sPow;
    const bool useLds = P.triPadded <= kLdsTris;
    if (useLds) {
        for (int i = threadIdx.x; i < P.triPadded; i += kBlock)
            sTris[i] = P.tris[i];
    }
    sPow.fill(threadIdx.x);
    __syncthreads();
    sPow.attach(P.env);
    const DevTri *lds = useLds ? sTris : nullptr;

    /* this wave's primary candidates (rtc_tile_cull) */
    const unsigned long long *tmask = nullptr;
    unsigned listLen = (unsigned)P.triCount;
    if (P.tileMask) {
        tmask = P.tileMask + (size_t)wave_tile(bx, by) * P.maskWords;
        listLen = 0;
        for (int w = 0; w < P.maskWords; ++w)
            listLen += (unsigned)__popcll(tmask[w]);
    }

    V3 acc{0.f, 0.f, 0.f};
    bool alive = valid && P.spp > 0 && P.maxBounce > 0;
    if (DEBUG && valid && !(P.maxBounce > 0)) {
        /* calcDebugColor with no bounce loop returns lerp(BLACK, WHITE, 0 / (float)maxBounce) */
        const float t = 0.f / (float)P.maxBounce;
        const V3 g = lerp(V3{0.f, 0.f, 0.f}, V3{1.f, 1.f, 1.f}, t);
        for (int i = 0; i < P.spp; ++i)
            acc = add(acc, mul(g, P.invSpp));
    }
    int sample = 0, bounce = 0;
    V3 pos = P.origin, dir = pdir, rayColor{1.f, 1.f, 1.f}, light{0.f, 0.f, 0.f};
    unsigned segCalls = 0, segTraced = 0;
    unsigned long long segTests = 0;

    /* Sky tile (wave-uniform): no triangle is a primary candidate anywhere in this 8x8 tile and there are
     * no spheres, so calculateRayCollision over the tile's (empty) candidate list misses for every primary
     * ray here, and every sample of calcColor is that one miss: light = 0 + env(dir) * (1,1,1)
     * (raytracing.c:268-293), acc += light * (float)(1/spp) (main.c:99).  Same operations as the state
     * machine below, without its per-segment bookkeeping; the sample loop is unrolled for ILP. */
    const bool skyTile = !DEBUG && !SPHERES && P.tileMask && listLen == 0;
    if (skyTile) {
        if (alive) {
#pragma unroll 2
            for (int s = 0; s < P.spp; ++s) {
                const V3 l = add(V3{0.f, 0.f, 0.f}, mulv(environment(pdir, P.env), V3{1.f, 1.f, 1.f}));
                acc = add(acc, mul(l, P.invSpp));
            }
            segCalls = (unsigned)P.spp;
            segTraced = P.hoist ? 1u : (unsigned)P.spp;
        }
        alive = false;
    }

    /* bit-exact primary-hit hoisting: the primary ray consumes no RNG, so its closest hit
     * is a function of the pixel; trace it once instead of once per sample. */
    Closest primary{999999.f, -1};
    if (P.hoist && alive) {
        primary = closest_hit<SPHERES>(P, pos, dir, true, tmask, lds);
        segTraced++;
        segTests += listLen;
    }

    while (__any(alive)) {
#ifdef RTC_DIAG
        diagIters++;
#endif
        /* wave-uniform: every live lane that traces this iteration is at bounce 0 (origin = camera) */
        const bool needTrace = alive && !(P.hoist && bounce == 0);
        const bool primaryWave = __all(!needTrace || bounce == 0);
        if (alive) {
            Closest c;
            segCalls++;
            if (!needTrace) {
                c = primary;
            } else {
#ifdef RTC_DIAG
                const unsigned long long dt0 = __builtin_amdgcn_s_memtime();
#endif
                c = closest_hit<SPHERES>(P, pos, dir, primaryWave, tmask, lds);
#ifdef RTC_DIAG
                diagTrace += __builtin_amdgcn_s_memtime() - dt0;
#endif
                segTraced++;
                segTests += primaryWave ? listLen : (unsigned)P.triCount;
            }
            bool endSample;
            if (c.idx >= 0) {
                /* closest.hitPoint = ray.pos + ray.dir * closest.dst (raytracing.c:238) */
                const V3 hitPoint = add(pos, mul(dir, c.dst));
                V3 normal, color;
                float emission, smoothness;
                if (SPHERES && c.idx < P.sphereCount) {
                    const DevSphere sp = P.spheres[c.idx];
                    normal = normalized(sub(hitPoint, V3{sp.cx, sp.cy, sp.cz})); /* raytracing.c:182 */
                    color = V3{sp.r, sp.g, sp.b};
                    emission = sp.emission;
                    smoothness = sp.smoothness;
                } else {
                    const int t = c.idx - (SPHERES ? P.sphereCount : 0);
                    const DevTri T = P.tris[t];
                    const DevMat M = P.mats[t];
                    normal = V3{T.nx, T.ny, T.nz};
                    color = V3{M.r, M.g, M.b};
                    emission = M.emission;
                    smoothness = M.smoothness;
                }
                /* calcColor hit branch, raytracing.c:274-287 (calcDebugColor :251-254 shares the first part) */
                const V3 diffuseDir = normalized(add(normal, random_direction(rng)));
                const V3 specularDir = reflect(dir, normal);
                dir = lerp(diffuseDir, specularDir, smoothness);
                pos = hitPoint;
                if (DEBUG) {
                    bounce++;
                    endSample = bounce >= P.maxBounce;
                    if (endSample)
                        light = lerp(V3{0.f, 0.f, 0.f}, V3{1.f, 1.f, 1.f}, (float)bounce / (float)P.maxBounce);
                } else {
                const V3 emitted = mul(color, emission);
                light = add(light, mulv(emitted, rayColor));
                rayColor = mulv(rayColor, color);
                const float p = fmax_ref(fmax_ref(rayColor.x, rayColor.y), rayColor.z);
                endSample = p < random_value(rng);
                if (!endSample) {
                    rayColor = mul(rayColor, rcp_cr(p)); /* (float)(1.0 / p) */
                    bounce++;
                    endSample = bounce >= P.maxBounce;
                }
                }
            } else if (DEBUG) {
                /* calcDebugColor: first miss ends the sample with lerp(BLACK, WHITE, i / (float)maxBounce) */
                light = lerp(V3{0.f, 0.f, 0.f}, V3{1.f, 1.f, 1.f}, (float)bounce / (float)P.maxBounce);
                endSample = true;
            } else {
                /* miss branch, raytracing.c:291 */
                light = add(light, mulv(environment(dir, P.env), rayColor));
                endSample = true;
            }
            if (endSample) {
                /* main.c:99: acc = acc + calcColor(...) * (float)(1./spp) */
                acc = add(acc, mul(light, P.invSpp));
                sample++;
                if (sample >= P.spp) {
                    alive = false;
                } else {
                    pos = P.origin;
                    dir = pdir;
                    rayColor = V3{1.f, 1.f, 1.f};
                    light = V3{0.f, 0.f, 0.f};
                    bounce = 0;
                }
            }
        }
    }

    if (valid) {
        const size_t o = (size_t)r * (size_t)P.width + (size_t)x;
        /* vec3ToColor (raytracing.c:11-15) fused */
        P.colors[3 * o] = float_to_u8(acc.x);
        P.colors[3 * o + 1] = float_to_u8(acc.y);
        P.colors[3 * o + 2] = float_to_u8(acc.z);
        if (P.accum) {
            P.accum[3 * o] = acc.x;
            P.accum[3 * o + 1] = acc.y;
            P.accum[3 * o + 2] = acc.z;
        }
    }
#ifdef RTC_DIAG
    if (g_rtc_diag && lane == 0) {
        const int wave = threadIdx.x >> 6;
        const size_t w = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (kBlock / 64) + wave;
        g_rtc_diag[4 * w] = __builtin_amdgcn_s_memtime() - diagT0;
        g_rtc_diag[4 * w + 1] = diagIters;
        g_rtc_diag[4 * w + 2] = diagT0;
        g_rtc_diag[4 * w + 3] = diagTrace;
    }
#endif
    flush_counters(P, segCalls, segTraced, segTests, lane);
}

/* LDS writes of this wave visible to its other lanes (the wave is the only user of the region) */
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* The sky pass (rtc_render_sky_rows): every pixel whose primary ray provably misses, few registers, so many waves per SIMD
 * hide the latency of the environment's double-precision chains.  <= 64 VGPRs: two sky waves fit where one chain wave
 * retires (frame -1.5 %, round 4). */
#ifndef RTC_SKY_WAVES
#define RTC_SKY_WAVES 8
#endif
/* Sky pixels by row strips (round 5): each wave takes 64 consecutive pixels of one launch row (workgroups of
 * kSkyWaves waves: kSkyWaves consecutive rows), so a strip of Color is 192 B = three whole 64-B lines when the row starts
 * on a line (every BASELINE width: 1920 * 3 and 3840 * 3 are multiples of 64), written by twelve 16-B stores staged in
 * LDS.  The 8x8-tile waves wrote 24-B tile rows that straddle lines shared with the neighbouring tiles' waves, so every
 * line was written back partially two or three times (sky WRITE_SIZE 12.0 MB per 1080p launch for 6.0 MB of Color,
 * VERDICT r04 #5).  A strip holding geometry pixels (rtc_render_chain writes those, maybe concurrently) or cut by the frame
 * edge writes its sky pixels' bytes only.  Same pixels, same per-sample environment loop, same values.  kSkyWaves waves per
 * workgroup: 1, or 4 for small shares of more than 400 k pixels (one-wave workgroups fill the registers and wave slots
 * the co-resident chain workgroups leave free at a finer grain -- whole frames -1 %, the 1080p 1/8 share -2 % -- but
 * the 1/4 share took 3.5 % longer with them, profiles/r04_zd_ab_sky_wg.log). */
/* GENERAL (round 6): the launch may merge (P.geoColor), hoist, write the accumulator or count segments; the pipelined
 * faithful whole frames run an instantiation without that code (56 VGPRs and no SGPR spill instead of 59 and 8). */
template <int kSkyWaves, bool GENERAL>
__global__ __launch_bounds__(kSkyWaves * 64) __attribute__((amdgpu_waves_per_eu(RTC_SKY_WAVES))) void rtc_render_sky_rows(
    RenderParams P)
{
    static_assert(kSkyWaves == 4 || kSkyWaves == 1, "one or four row strips per workgroup");
    __shared__ PowTablesLds sPow;
    __shared__ __attribute__((aligned(16))) unsigned char sStrip[kSkyWaves][192];
    sPow.fill(threadIdx.x);
    __syncthreads();
    sPow.attach(P.env);
    const int lane = threadIdx.x & 63, lw = threadIdx.x >> 6;
    unsigned segCalls = 0, segTraced = 0;
    const int r = (int)blockIdx.y * kSkyWaves + __builtin_amdgcn_readfirstlane(lw); /* launch row (wave-uniform) */
    const int x = (int)blockIdx.x * 64 + lane;
    const bool inFrame = r < P.rows && x < P.width;
    /* the pixel's tile: pixels with a primary candidate are rtc_render_chain's (pixMask bit (row % 8) * 8 + x % 8) */
    bool geo = false;
    int t = 0;
    if (inFrame) {
        t = (r >> 3) * (P.blocksX * 2) + (x >> 3);
        geo = ((P.pixMask[t] >> (((r & 7) << 3) | (x & 7))) & 1ull) != 0ull;
    }
    const bool valid = inFrame && !geo; /* a sky pixel: this kernel renders it */
    /* merged (P.geoColor): the geometry kernel has finished; its pixels' bytes are written here too, so every strip is
     * whole lines.  Their words are requested now and used after the sky loop. */
    const bool merged = GENERAL && P.geoColor != nullptr; /* (uniform) */
    const bool writes = merged ? inFrame : valid;
    const unsigned long long mine = __ballot(writes);
    if (mine == 0ull)
        return;
    unsigned gw = 0;
    if (merged) {
        /* the geometry kernel's items are the sub-lists concatenated: entry pos of sub-list l is item (entries of the
         * sub-lists before l) + pos -- the exclusive prefix of the launch's counts, lane l holding sub-list l's */
        const int cnt = lane < kGeoLists ? min(P.geoCount[lane * kGeoCountStride], P.geoCap) : 0;
        int incl = cnt;
#pragma unroll
        for (int d = 1; d < kGeoLists; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d)
                incl += v;
        }
        const unsigned e = geo ? P.pixItem[(size_t)t * 64 + (((r & 7) << 3) | (x & 7))] : 0u;
        const int excl = __shfl(incl - cnt, (int)(e % kGeoLists));
        if (geo)
            gw = P.geoColor[excl + (int)(e / kGeoLists)];
    }
    const int y = launch_row_y(P, r);
    const V3 dir = primary_dir(P, x, y);
    V3 acc{0.f, 0.f, 0.f};
    if (valid && P.spp > 0 && P.maxBounce > 0) {
        /* hoisted mode evaluates the primary ray's miss once (a function of the pixel, like its closest hit), faithful
         * mode every sample */
        if (GENERAL && P.hoist) {
            const V3 l = add(V3{0.f, 0.f, 0.f}, mulv(environment(dir, P.env), V3{1.f, 1.f, 1.f}));
            for (int s = 0; s < P.spp; ++s)
                acc = add(acc, mul(l, P.invSpp));
        } else {
            /* the sun term provably below half an ulp of every colour component for this pixel (sun_vanishes, a
             * function of the pixel's direction and the launch's environment) */
            const bool vanish = sun_vanishes(dir, P.env);
#pragma unroll 2
            for (int s = 0; s < P.spp; ++s) {
#if defined(RTC_AB_CHEAP_ENV_SKY) && defined(RTC_EXPERIMENT) /* timing experiment only (the environment's cost) */
                const V3 l = lerp(P.env.horizon, P.env.zenith, fmaxf(dir.y + (float)s * 1e-9f, 0.f));
#else
                /* raytracing.c:291 with rayColor (1, 1, 1): 0 + environment (environment_miss_term: acc starts at +0) */
                const V3 l = environment_miss_term(dir, P.env, vanish);
#endif
                acc = add(acc, mul(l, P.invSpp)); /* main.c:99 */
            }
        }
        segCalls = (unsigned)P.spp;
        segTraced = P.hoist ? 1u : (unsigned)P.spp;
    }
    /* vec3ToColor (raytracing.c:11-15, main.c:101); a geometry pixel's bytes as the geometry kernel quantised them */
    const unsigned char c0 = valid ? float_to_u8(acc.x) : (unsigned char)(gw & 0xffu);
    const unsigned char c1 = valid ? float_to_u8(acc.y) : (unsigned char)((gw >> 8) & 0xffu);
    const unsigned char c2 = valid ? float_to_u8(acc.z) : (unsigned char)((gw >> 16) & 0xffu);
    unsigned char *const rowp = P.colors + 3 * ((size_t)r * (size_t)P.width + (size_t)blockIdx.x * 64);
    const bool whole = mine == ~0ull && ((uintptr_t)rowp & 15u) == 0u; /* wave-uniform */
    if (whole) {
        unsigned char *st = sStrip[lw];
        st[3 * lane] = c0;
        st[3 * lane + 1] = c1;
        st[3 * lane + 2] = c2;
        wave_lds_sync();
        if (lane < 12)
            ((uint4 *)rowp)[lane] = ((const uint4 *)st)[lane];
    } else if (writes) {
        rowp[3 * lane] = c0;
        rowp[3 * lane + 1] = c1;
        rowp[3 * lane + 2] = c2;
    }
    if (GENERAL && valid && P.accum) {
        const size_t o = 3 * ((size_t)r * (size_t)P.width + (size_t)x);
        P.accum[o] = acc.x;
        P.accum[o + 1] = acc.y;
        P.accum[o + 2] = acc.z;
    }
    if (GENERAL)
        flush_counters(P, segCalls, segTraced, 0ull, lane);
}

/* ---- state-indexed samples (rtc_render_chain, the default for pixels that see geometry) --------------------
 * A pixel's samples are chained only through its RNG state (main.c:95-100), and in the OBJ scenes every sample
 * whose primary ray hits draws exactly 7 values per hit (RandomDiretion's six, moremath.c:104-108, and the
 * roulette draw, raytracing.c:285) and none on a miss.  So a sample is a pure function of the draw offset it
 * starts at: write S_j for the sample started from the seed advanced by 7 j draws (rng_advance; the LCG step
 * is affine) and h_j for its number of hits.  The reference's k-th sample is S_{j_k} with
 *     j_0 = 0,   j_{k+1} = j_k + h_{j_k}
 * (h >= 1 when the primary ray hits; when it misses every sample is S_0 and h = 0).  The kernel evaluates
 * S_j for a window of consecutive j -- one lane per j, 64 at a time -- and then walks the chain through the
 * window, adding the members' radiance in sample order (main.c:99, sequential f32 adds).  Every accumulated
 * value is one of the reference's samples, computed by the reference's operations from its exact start state,
 * so the frame is bit-identical; no prediction is involved.  ~97 % of the geometry pixels of the BASELINE frame
 * have no sample with a second hit (sum h = spp), so one window of 64 covers them; the others take a second
 * window.  The lanes of a wave share the pixel's primary ray: the primary trace is wave-uniform (scalar-loaded
 * candidate records), the shading at the primary hit runs in lockstep, and only the bounce segments diverge.
 * Work: one wave per geometry pixel, from the tile cull's sub-lists (see the kernel). */
static_assert(sizeof(SampleSlot) == rtcplan::kSampleSlotBytes, "the planner sizes the deferred sample slots");
/* Shares (row stride > 1) of up to rtcplan::kInlineSumPixels pixels are "small": they sum in-kernel and,
 * pipelined, prepare, cull and run their geometry kernel on the two cull streams.  Round 4 raised it
 * from 400 k to 600 k pixels so that the 1080p 1/4 share (518 k) is one: 0.137 -> 0.117 ms per pipelined share; the
 * 1/2 share and the 4K 1/8 share (1.04 M) measured no better that way (tools/scale_probe.py, profiles/r04_y_*) */
#ifndef RTC_SUN_VANISH
#define RTC_SUN_VANISH 1 /* (A/B switch, round 6) */
#endif
#ifndef RTC_SKY_MERGE
#define RTC_SKY_MERGE 1 /* (A/B switch, round 6) */
#endif
constexpr int kChainBlock = 256; /* threads per chain workgroup (two-wave workgroups were slower everywhere, r04_ze) */
/* Persistent chain workgroups per CU (each 4 waves of 128 VGPRs: 4 fill every SIMD's registers).  A whole frame runs 3,
 * so that a quarter of every SIMD's registers holds two sky waves (<= 64 VGPRs) from the start: the sky pass then runs
 * in the chain kernel's idle issue slots instead of waiting for its tail, and the launch stream's small kernels are no
 * longer starved by that tail (round 4: frame 0.372 -> 0.351 ms; 4 per CU: 0.370 vs 0.340 ms on the alternating streams,
 * though fsuzane, whose frame is nearly all geometry kernel, takes 1.12 vs 1.22 ms with 4).  Small shares run 3 too since
 * consecutive shares overlap on the alternating streams (4 before).  Round 5: whole frames of scenes whose bounce rays
 * often hit again run 4 (RTC_CHAIN_WGS_HIT, chosen at upload by bounce_hit_share).  Workers = per-CU count x CUs:
 * exactly the resident capacity, no second round.  (RTC_CHAIN_WGS_FULL / _HIT are defined with kSkySlots.) */
#ifndef RTC_CHAIN_WGS_SHARE
#define RTC_CHAIN_WGS_SHARE 3 /* 1/4 share 0.116 -> 0.113 ms, 1/8 share 0.075 -> 0.074 ms (round 4, r04_za) */
#endif
#ifndef RTC_CHAIN_WAVES
#define RTC_CHAIN_WAVES 4
#endif

/* The bounce segments of a wave's lanes (calculateRayCollision, raytracing.c:216-240), as a dense list of
 * (lane, cluster) pairs.  Each live lane culls the clusters its half-line cannot reach (DevCluster bound) and
 * enters the rest into the wave's pair list (cluster-major); the list is then processed 64 pairs at a time,
 * every lane taking one pair: the owner's ray from LDS, the cluster's 8 records from LDS (staged once per
 * workgroup), the exact-safe filter and the reference arithmetic for survivors.  A pair's closest hit goes
 * to its owner with an LDS atomic minimum on (dst bits << 32 | index): dst >= EPSILON > 0, so the float bits
 * order like the values and the key order is the lexicographic (dst, index) order -- the lowest index among
 * equal distances, as the reference's strict `<` over ascending indices keeps (raytracing.c:231).  Only
 * candidates with dst < 999999 (the reference's initial closest distance, raytracing.c:218) enter.
 * Compared with a wave-uniform loop over the union of the lanes' clusters (every lane masked through every
 * cluster some lane needs), each ray-triangle test here occupies one lane-slot instead of up to 64. */
typedef float f2 __attribute__((ext_vector_type(2)));
/* A sample's m-th hit draws the 7 values at state index j + m (RandomDiretion's six, the roulette's one): exactly
 * what S_{j+m}'s first hit draws.  So the window's active lanes enter the draws of their own state index, computed
 * at the primary hit, in a per-wave LDS table, and a later hit of lane l in bounce iteration i reads entry l + i
 * instead of running Box-Muller again; only lanes with l + i past the window's active lanes compute theirs (the
 * state advanced by 7 i draws).  The values are the same function of the same state, so the frame is unchanged;
 * what goes is most of the divergent Box-Muller passes of the bounce iterations with a hit (scenes whose rays hit
 * several times: fsuzane 2.00 -> 1.93 ms per frame, 1.77 with the dense culls below). */
constexpr int kChainPairs = 1024;
struct ChainWaveLds {
    float4 cl[kChunkClusters][2]; /* first bounces: the clusters' origin terms (ClusterTerms) */
    unsigned long long key[64];   /* closest hit per lane, (dst bits << 32) | index */
    /* lane | cluster << 6 (or lane | record << 6), cluster-major; a full list is run through the passes and
     * refilled.  Its size keeps a block (4 waves + the staged records of one chunk) within 40 KB of LDS: four
     * blocks per CU, the 4 waves per SIMD that 128 VGPRs allow */
    unsigned short pair[kChainPairs];
    float4 draw[64]; /* the window's hit draws by state index jn + i: RandomDirection's vector, the roulette value */
};
constexpr unsigned long long kNoHitKey = ((unsigned long long)0x497423F0u << 32) | 0xFFFFFFFFull; /* 999999.f */
static_assert(kChunkClusters <= 32, "cluster masks are 32-bit");
static_assert(kChainPairs >= 64 * kClusterSize, "one cluster's pairs of a full wave fit the list");
static_assert(kChainPairs * sizeof(unsigned short) >= 3 * 64 * sizeof(float), "a window's staged samples fit the list");
/* rtc_render_chain's static LDS (powf tables, the waves' ChainWaveLds, the work counter) and the block budget
 * that keeps 4 blocks (16 waves) per CU */
constexpr size_t kChainStaticLds = sizeof(PowTablesLds) +
                                   (kChainBlock / 64) * sizeof(ChainWaveLds) + 64 +
                                   kChunkClusters * sizeof(DevCluster) /* sCl (the dense culls) */;
constexpr size_t kCuLds = 160 * 1024; /* gfx950 LDS per CU */
/* the block LDS that keeps the chain workgroups per CU at most n: above kCuLds / (n + 1) */
constexpr size_t chain_lds_floor(int n) { return n >= 4 ? 0 : kCuLds / (size_t)(n + 1) + 256; }

/* The pair passes: entry i of W.pair (i < n) is a (lane, cluster) pair -- the cluster's 8 records; the owner's ray
 * by ds_bpermute from the owner lane (every lane takes part), the exact-safe filter, the reference arithmetic for
 * survivors, an atomic lexicographic minimum into the owner's key. */
/* The clustered records staged in LDS structure-of-arrays: 16-B quarter k of record i at q[k * n + i], n = the
 * staged record count.  Lanes reading different records then hit different banks in ds_read_b128's 16-lane
 * groups (64-B records at lane-varying indices put four lanes of a group on each bank); one record is still four
 * ds_read_b128.  (Round 5 tried a slot skipped after every cluster, for pair passes whose lanes read record j of
 * different clusters: conflict cycles 3.8 M -> 5.0 M per 1080p launch -- the pair list is cluster-major, so a pass's
 * lanes mostly share a cluster, while the reach table's consecutive records then straddled the skipped slots.) */
__host__ __device__ constexpr int soa_slots(int n) { return n; }
__device__ __forceinline__ DevTri rec_soa(const float4 *__restrict__ q, int n, int i)
{
    DevTri t;
    float4 *v = (float4 *)&t;
    v[0] = q[i];
    v[1] = q[n + i];
    v[2] = q[2 * n + i];
    v[3] = q[3 * n + i];
    return t;
}
__device__ __forceinline__ float bperm_f(int srcLane, float v)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(srcLane << 2, __float_as_int(v)));
}
template <bool MULTI>
__device__ __forceinline__ void chain_pair_passes(const RenderParams &P, int n, int c0, const float4 *__restrict__ sRec,
                                                  ChainWaveLds &W, int lane, V3 pos, V3 dir)
{
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        const unsigned pr = i < n ? W.pair[i] : (unsigned)lane;
        const int o = (int)(pr & 63u);
        const V3 rpos{bperm_f(o, pos.x), bperm_f(o, pos.y), bperm_f(o, pos.z)};
        const V3 rdir{bperm_f(o, dir.x), bperm_f(o, dir.y), bperm_f(o, dir.z)};
        if (i < n) {
            Closest c{999999.f, -1};
            const int r0 = (c0 + (int)(pr >> 6)) * kClusterSize, nRec = P.clusterCount * kClusterSize;
            auto rec = [&](int j) -> DevTri { return MULTI ? P.clTris[r0 + j] : rec_soa(sRec, nRec, r0 + j); };
            unsigned surv = 0;
#pragma unroll 4 /* (round 5: 4 vs 2, fsuzane -1 %, headline within noise; same registers) */
            for (int j = 0; j < kClusterSize; ++j)
                surv |= (unsigned)general_filter(rpos, rdir, rec(j)) << j;
            while (surv) {
                const int j = __builtin_ctz(surv);
                surv &= surv - 1;
                const DevTri R = rec(j);
                general_exact(rpos, rdir, R, __float_as_int(R.pad0), c);
            }
            if (c.idx >= 0 && c.dst < 999999.f)
                atomicMin(&W.key[o], ((unsigned long long)__float_as_uint(c.dst) << 32) | (unsigned)c.idx);
        }
    }
}
/* The first-bounce pairs as (lane, live cluster j) -- one entry per cluster a lane keeps, the pass
 * looping over that cluster's records reachable from p0 (W.cl[j][1]: z = cluster index, w = reach bits); one
 * atomic per entry instead of one per record */
__device__ __forceinline__ void chain_pair_passes_cl(int n, const float4 *__restrict__ sRec, int nRec, ChainWaveLds &W,
                                                     int lane, V3 pos, V3 dir)
{
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        const unsigned pr = i < n ? W.pair[i] : (unsigned)lane;
        const int o = (int)(pr & 63u);
        const V3 rpos{bperm_f(o, pos.x), bperm_f(o, pos.y), bperm_f(o, pos.z)};
        const V3 rdir{bperm_f(o, dir.x), bperm_f(o, dir.y), bperm_f(o, dir.z)};
        if (i < n) {
            const float4 kb = W.cl[pr >> 6][1];
            const int r0 = __float_as_int(kb.z) * kClusterSize;
            Closest c{999999.f, -1};
            for (unsigned r = (unsigned)__float_as_int(kb.w); r; r &= r - 1) {
                const DevTri T = rec_soa(sRec, nRec, r0 + __builtin_ctz(r));
                if (general_filter(rpos, rdir, T))
                    general_exact(rpos, rdir, T, __float_as_int(T.pad0), c);
            }
            if (c.idx >= 0 && c.dst < 999999.f)
                atomicMin(&W.key[o], ((unsigned long long)__float_as_uint(c.dst) << 32) | (unsigned)c.idx);
        }
    }
}

/* Dense cluster culls (single-chunk scenes, bounce segments after the first): with a live lanes and nCl clusters, the
 * per-lane loop issues nCl culls for the wave however few lanes are live; instead the wave takes the a * nCl (live
 * lane, cluster) culls 64 at a time -- cluster-major, so the pairs kept come out in the per-lane loop's order -- the
 * owner's ray by ds_bpermute, the cluster from LDS.  Taken while a <= kDenseCullMax (fsuzane 1.93 -> 1.77 ms per
 * frame with 16, 1.80 with 32; the headline frame, whose later bounces are rare, within noise). */
constexpr int kDenseCullMax = 16;
static_assert(kDenseCullMax * kChunkClusters <= kChainPairs, "a dense cull's pairs fit the list");
static_assert(sizeof(ChainWaveLds::cl) >= 64 * sizeof(int), "the dense cull's owner lanes fit W.cl");

template <bool MULTI, bool COUNT, bool HITS>
__device__ __forceinline__ Closest chain_trace_pairs(const RenderParams &P, bool alive, bool firstBounce, V3 pos,
                                                     V3 dir, const float4 *__restrict__ sRec, ChainWaveLds &W,
                                                     int lane, unsigned &tests, const DevCluster *__restrict__ sCl)
{
    W.key[lane] = kNoHitKey;
    const float rho = fabsf(dir.x) + fabsf(dir.y) + fabsf(dir.z), dd = dir_dd(dir);
    const bool rhoOk = P.clusterCull && rho <= kClusterRhoMax;
    tests = 0;
    /* A pixel's first bounces all start at its primary hit point p0 (lane 0's pos; single-chunk scenes):
     *  - the clusters' origin terms, once, one lane per cluster, into LDS, compacted to the clusters with a
     *    record reachable from p0 (below), so the per-lane cull loop is branch-free over those only;
     *  - the records that can be hit from p0 at all, one lane per record: the reference's own f32
     *    dot(AC, (p0 - A) x AB) > 0, or a stored normal not aligned with the geometric one (aligned_normal:
     *    with an aligned normal and that dot <= 0, rayTriangle rejects every direction from p0).
     * The records that cannot be hit are not tested; the rest are tested as (lane, record) pairs.  The argument
     * holds for |dir|_1 <= kClusterRhoMax: a wave with a live ray beyond that takes the per-cluster path. */
    const bool table = !MULTI && firstBounce && P.clusterCull && !__ballot(alive && !rhoOk);
    unsigned long long reach[kChunkClusters * kClusterSize / 64];
    unsigned long long live = 0; /* clusters with a record reachable from p0 (their terms compacted in W.cl) */
    DSECT_BEGIN(dtab);
    if (table) {
        const V3 p0{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(pos.x), 0)),
                    __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pos.y), 0)),
                    __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pos.z), 0))};
#pragma unroll
        for (int q = 0; q < kChunkClusters * kClusterSize / 64; ++q) {
            const int i = q * 64 + lane;
            bool can = false;
            if (i < P.clusterCount * kClusterSize) {
                const DevTri R = rec_soa(sRec, P.clusterCount * kClusterSize, i);
                if (__float_as_int(R.pad0) >= 0) {
                    const V3 sv = sub(p0, V3{R.ax, R.ay, R.az});               /* raytracing.c:198 */
                    const V3 qv = cross(sv, V3{R.abx, R.aby, R.abz});          /* :202 */
                    const float dac = dot(V3{R.acx, R.acy, R.acz}, qv);        /* :206 numerator */
                    can = dac > 0.f || __float_as_int(R.pad1) == 0;
                }
            }
            reach[q] = __ballot(can);
        }
        /* lane k < clusterCount: cluster k's reachable records r8; the clusters with any enter W.cl compacted, in
         * cluster order, with (k, r8) in the second vector */
        unsigned r8l = 0;
        if (lane < P.clusterCount) {
            const unsigned long long rw = lane < 8 ? reach[0] : lane < 16 ? reach[1] : lane < 24 ? reach[2] : reach[3];
            r8l = (unsigned)(rw >> ((lane & 7) * 8)) & 0xffu;
        }
        live = __ballot(r8l != 0u);
        if (r8l) {
            const int pos = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(live >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((unsigned)live, 0u));
            /* (the workgroup's LDS copy of the clusters: a global load here was a round trip on every window) */
            const ClusterTerms t = cluster_terms(p0, sCl[lane]);
            W.cl[pos][0] = make_float4(t.w.x, t.w.y, t.w.z, t.w2);
            W.cl[pos][1] = make_float4(t.A, t.B, __int_as_float(lane), __int_as_float((int)r8l));
        }
        wave_lds_sync();
    }
    DSECT_END(dtab, 14);
    /* scenes of more than kChunkClusters clusters: chunk by chunk (a chunk's ball culls its clusters for a lane
     * at once); the records come from global memory when they are not staged in LDS (sRec null) */
    const int nChunks = MULTI ? P.chunkCount : 1;
    for (int h = 0; h < nChunks; ++h) {
        const int c0 = h * kChunkClusters, nCl = MULTI ? min(kChunkClusters, P.clusterCount - c0) : P.clusterCount;
        bool in = alive;
        if (MULTI) {
            if (alive)
                in = !(rhoOk && cluster_culled(pos, dir, rho, dd, P.chunks[h]));
            if (!__ballot(in))
                continue;
        }
        unsigned cm = 0;
        int n = 0;
        DSECT_BEGIN(dc3);
        const unsigned long long inM = __ballot(in);
        const int nIn = (int)__popcll(inM);
        const bool dense = !MULTI && !table && nIn <= kDenseCullMax;
        if (dense) {
            int *own = (int *)&W.cl[0][0]; /* W.cl is free outside the first bounce's table mode */
            int *kept = own + 64;          /* COUNT: per owner lane, clusters kept (+ 1 << 16 for the scene's last) */
            if (in)
                own[__builtin_amdgcn_mbcnt_hi((unsigned)(inM >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)inM, 0u))] = lane;
            if (COUNT)
                kept[lane] = 0;
            wave_lds_sync();
            const int tot = nIn * nCl;
            const unsigned magic = nIn > 1 ? (unsigned)((0x100000000ull + (unsigned)nIn - 1u) / (unsigned)nIn) : 0u;
            for (int b = 0; b < tot; b += 64) {
                const int e = b + lane;
                const int k = nIn > 1 ? (int)__umulhi((unsigned)e, magic) : e; /* e / nIn, exact for e < 2^16 */
                const bool valid = e < tot;
                const int o = own[valid ? e - k * nIn : 0];
                const V3 rp{bperm_f(o, pos.x), bperm_f(o, pos.y), bperm_f(o, pos.z)};
                const V3 rd{bperm_f(o, dir.x), bperm_f(o, dir.y), bperm_f(o, dir.z)};
                bool keep = false;
                if (valid) {
                    const float rr = fabsf(rd.x) + fabsf(rd.y) + fabsf(rd.z);
                    keep = !(P.clusterCull && rr <= kClusterRhoMax && cluster_culled(rp, rd, rr, dir_dd(rd), sCl[k]));
                }
                const unsigned long long m = __ballot(keep);
                if (keep)
                    W.pair[n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                        (unsigned short)(o | (k << 6));
                if (COUNT && keep)
                    atomicAdd(&kept[o], 1 + (k == P.clusterCount - 1 ? 1 << 16 : 0));
                n += (int)__popcll(m);
            }
            if (COUNT) {
                wave_lds_sync();
                const int kc = kept[lane];
                tests = (unsigned)(kc & 0xffff) * kClusterSize -
                        (unsigned)(kc >> 16) * (unsigned)(P.clusterCount * kClusterSize - P.triCount);
            }
        }
        /* table mode: bit j of cm = the j-th live cluster kept (branch-free body over the compacted terms) */
        const int nLive = __popcll(live);
        /* (round 6) table mode with every lane's pairs fitting the list: the cull and the pair list in one pass over the
         * live clusters -- each cluster's ballot of the lanes keeping it appends their entries at once, in the same
         * cluster-major, lane-ascending order as the separate build below (frame -0.7 %, profiles/r06_p_ab_fused_pairs.log) */
        const bool fused = table && nLive * 64 <= kChainPairs; /* (uniform) */
        /* the same for the per-lane culls of later bounces (more than kDenseCullMax live lanes), in the HITS instantiation
         * only: fsuzane -1 to -2 %, while in the one instantiation of round 6's first try the headline's geometry kernel --
         * which never takes that path -- took 0.8-1.4 % longer from the code it adds (profiles/r06_t / r06_u / r06_v) */
        const bool fusedG = HITS && !firstBounce && !table && !dense && nCl * 64 <= kChainPairs; /* (uniform) */
        if (fusedG) {
            for (int k = 0; k < nCl; ++k) {
                const bool kept = in && !(rhoOk && cluster_culled(pos, dir, rho, dd, P.clusters[c0 + k]));
                cm |= (unsigned)kept << k;
                const unsigned long long m = __ballot(kept);
                if (kept)
                    W.pair[n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                        (unsigned short)(lane | (k << 6));
                n += (int)__popcll(m);
            }
            if (in) /* triangles in the clusters kept (only the scene's last cluster has zero records) */
                tests += (unsigned)__popc(cm) * kClusterSize -
                         (c0 + nCl == P.clusterCount ? ((cm >> (nCl - 1)) & 1u) : 0u) *
                             (unsigned)(P.clusterCount * kClusterSize - P.triCount);
        } else if (fused) {
#pragma unroll 4
            for (int j = 0; j < nLive; ++j) {
                const float4 a = W.cl[j][0], b = W.cl[j][1];
                const ClusterTerms t{V3{a.x, a.y, a.z}, a.w, b.x, b.y};
                const bool kept = in && !(rhoOk && culled_by(t, dir, rho, dd));
                tests += kept ? (unsigned)__popc((unsigned)__float_as_int(b.w)) : 0u;
                const unsigned long long m = __ballot(kept);
                if (kept)
                    W.pair[n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                        (unsigned short)(lane | (j << 6));
                n += (int)__popcll(m);
            }
        } else if (dense) {
        } else if (in && table) {
            /* (round 6: each live cluster's terms by v_readlane from the lane that computed them instead of these LDS
             * reads -- six VALU readlanes per cluster: chain kernel +3 %, frame +2.4 %, profiles/r06_c_ab_*) */
#pragma unroll 4
            for (int j = 0; j < nLive; ++j) {
                const float4 a = W.cl[j][0], b = W.cl[j][1];
                const ClusterTerms t{V3{a.x, a.y, a.z}, a.w, b.x, b.y};
                const bool kept = !(rhoOk && culled_by(t, dir, rho, dd));
                cm |= (unsigned)kept << j;
                tests += kept ? (unsigned)__popc((unsigned)__float_as_int(b.w)) : 0u;
            }
        } else if (in) {
            for (int k = 0; k < nCl; ++k)
                cm |= (unsigned)!(rhoOk && cluster_culled(pos, dir, rho, dd, P.clusters[c0 + k])) << k;
            /* triangles in the clusters kept (only the scene's last cluster has zero records) */
            tests += (unsigned)__popc(cm) * kClusterSize -
                     (c0 + nCl == P.clusterCount ? ((cm >> (nCl - 1)) & 1u) : 0u) *
                         (unsigned)(P.clusterCount * kClusterSize - P.triCount);
        }
        DSECT_END(dc3, 3);
        DSECT_BEGIN(dc4);
        constexpr int kCap = kChainPairs;
        if (dense || fused || fusedG) {
        } else if (table) {
            /* (lane, live cluster) entries, one per cluster a lane keeps; the list is flushed through the passes
             * whenever the next cluster would overflow it */
            for (int j = 0; j < nLive; ++j) {
                const unsigned long long m = __ballot((cm >> j) & 1u);
                if (!m)
                    continue;
                if (n + (int)__popcll(m) > kCap) {
                    wave_lds_sync();
                    chain_pair_passes_cl(n, sRec, P.clusterCount * kClusterSize, W, lane, pos, dir);
                    wave_lds_sync();
                    n = 0;
                }
                if ((cm >> j) & 1u)
                    W.pair[n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                        (unsigned short)(lane | (j << 6));
                n += (int)__popcll(m);
            }
        } else {
            for (int k = 0; k < nCl; ++k) {
                const unsigned long long m = __ballot((cm >> k) & 1u);
                if (!m)
                    continue;
                if (n + (int)__popcll(m) > kCap) {
                    wave_lds_sync();
                    chain_pair_passes<MULTI>(P, n, c0, sRec, W, lane, pos, dir);
                    wave_lds_sync();
                    n = 0;
                }
                if ((cm >> k) & 1u)
                    W.pair[n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                        (unsigned short)(lane | (k << 6));
                n += (int)__popcll(m);
            }
        }
        wave_lds_sync();
        DSECT_END(dc4, 4);
        DSECT_BEGIN(dc5);
        if (table)
            chain_pair_passes_cl(n, sRec, P.clusterCount * kClusterSize, W, lane, pos, dir);
        else
            chain_pair_passes<MULTI>(P, n, c0, sRec, W, lane, pos, dir);
        wave_lds_sync(); /* the pair list is rewritten by the next chunk */
        DSECT_END(dc5, 5);
    }
    const unsigned long long key = W.key[lane];
    Closest c{999999.f, -1};
    if (key != kNoHitKey) {
        c.dst = __uint_as_float((unsigned)(key >> 32));
        c.idx = (int)(unsigned)key;
    }
    return c;
}

/* The deferred half of rtc_render_chain's walk: for each geometry pixel with a slot, its accumulated samples'
 * radiance in sample order (main.c:97-100: acc = acc + calcColor(...) * (1/spp), sequential f32 adds from 0), then
 * vec3ToColor (raytracing.c:11-15).  One lane per pixel.  (Summing a wave's own pixels at the end of
 * rtc_render_chain instead, without this launch, measured 0.477 vs 0.430 ms per frame: the waves' serial tails hold
 * their CUs while the sky pass waits for them.) */
__global__ __launch_bounds__(256) void rtc_accumulate_samples(RenderParams P)
{
    int items = 0;
    for (int l = 0; l < kGeoLists; ++l)
        items += min(P.geoCount[l * kGeoCountStride], P.geoCap);
    items = min(items, P.sampleCap);
    for (int it = blockIdx.x * 256 + threadIdx.x; it < items; it += gridDim.x * 256) {
        const SampleSlot *slot = P.sampleBuf + (size_t)it * (size_t)P.spp;
        f2 accxy{0.f, 0.f};
        float accz = 0.f;
        if (P.maxBounce > 0) {
#pragma unroll 8
            for (int k = 0; k < P.spp; ++k) {
                const SampleSlot v = slot[k];
                accxy = accxy + f2{v.x, v.y};
                accz = accz + v.z;
            }
        }
        const size_t o = (size_t)P.itemPix[it];
        P.colors[3 * o] = float_to_u8(accxy.x);
        P.colors[3 * o + 1] = float_to_u8(accxy.y);
        P.colors[3 * o + 2] = float_to_u8(accz);
        if (P.accum) {
            P.accum[3 * o] = accxy.x;
            P.accum[3 * o + 1] = accxy.y;
            P.accum[3 * o + 2] = accz;
        }
    }
}

/* Primary segments over the tile's candidates (rtc_render_chain) with the filter records staged in LDS (null: from
 * global memory): the filter's record is an LDS read instead of a dependent scalar load per candidate; DevPrimX
 * (survivors only) stays global.  Same operations as closest_primary_listed. */
__device__ __forceinline__ void closest_primary_listed_lds(const RenderParams &P, V3 dir, Closest &c, const unsigned long long *__restrict__ mask,
                                                           unsigned long long m0, unsigned long long m1,
                                                           const DevPrimF *__restrict__ sF, bool staged)
{
    /* m0, m1: the tile's first two mask words, already read (the chain kernel prefetches them one item ahead) */
    const int maskWords = KARG(maskWords);
    const DevPrimF *const primF = KARG(primF);
    const DevPrimX *const primX = KARG(primX);
    for (int w = 0; w < maskWords; ++w) {
        unsigned long long m = w == 0 ? m0 : w == 1 ? m1 : KCONST(mask)[w];
        while (m) {
            const int t = w * 64 + __builtin_ctzll(m);
            m &= m - 1;
            /* two loads of known address space (LDS, or a scalar load): a pointer that may be either would be
             * read with flat loads, whose wait also covers the wave's pending slot stores.  (Requesting the next
             * candidate's record before testing this one, round 6: 1080p shares 2-3 % longer, the frame unchanged,
             * profiles/r06_i_ab_cull_trim_xcd_runs_prefetch.log.) */
            const DevPrimF F = staged ? sF[t] : KLOAD(primF, t);
            if (!prim_backfacing(dir, F) && prim_pass(dir, F) && !(dot(dir, V3{F.nx, F.ny, F.nz}) >= 0.f)) {
                /* the reference's arithmetic (raytracing.c:189-208) */
                const DevPrimX X = KLOAD(primX, t);
                const V3 h = cross(dir, V3{X.acx, X.acy, X.acz});
                const float det = dot(V3{X.abx, X.aby, X.abz}, h);
                if (!(-kEps < det && det < kEps)) {
                    const float invDet = rcp_cr(det); /* IEEE 1.f / det */
                    const float u = dot(V3{X.s0x, X.s0y, X.s0z}, h) * invDet;
                    const float v = dot(dir, V3{X.q0x, X.q0y, X.q0z}) * invDet;
                    const float dst = X.dac0 * invDet;
                    if (!(u < 0.f || u > 1.f) && !(v < 0.f || u + v > 1.f) && !(dst < kEps) && dst < c.dst) {
                        c.dst = dst;
                        c.idx = t;
                    }
                }
            }
        }
    }
}

/* rtc_render_chain's dynamic LDS: the clustered records (MULTI: none), then, when the block's budget allows
 * (P.chainPrimF), the primary filter records.  (Staging the primary exact records and the shading records as well
 * measured no faster.) */
struct ChainStage {
    float4 *rec; /* structure-of-arrays (rec_soa) */
    DevPrimF *primF;
};
template <bool MULTI>
__device__ __forceinline__ ChainStage chain_stage(const RenderParams &P, unsigned char *sDyn)
{
    ChainStage S{nullptr, nullptr};
    if (!MULTI)
        S.rec = (float4 *)sDyn;
    if (P.chainPrimF)
        S.primF = (DevPrimF *)(sDyn + (MULTI ? 0 : (size_t)soa_slots(P.clusterCount * kClusterSize) * sizeof(DevTri)));
    const int nRec = P.clusterCount * kClusterSize, slots = soa_slots(nRec);
    for (int i = threadIdx.x; S.rec && i < nRec; i += kChainBlock) {
        const float4 *g = (const float4 *)(P.clTris + i);
        for (int k = 0; k < 4; ++k)
            S.rec[k * slots + i] = g[k];
    }
    for (int i = threadIdx.x; S.primF && i < P.triPadded; i += kChainBlock)
        S.primF[i] = P.primF[i];
    return S;
}

/* COUNT: the launch asks for segment counters (instrumentation, untimed); without it the counters are compiled out */
/* MULTI: more than one chunk of clusters (chunk-level culling, records from global).  GENERAL (round 6): the launch may give
 * items deferred sample slots (P.sampleCap > 0: joined whole frames), hoist the primary segments (P.hoist) or read the
 * primary filter records from global memory (!P.chainPrimF: too large to stage); without it every item sums in-kernel
 * and traces its primary ray per sample over the staged records, and none of the other code is in the kernel -- the pipelined faithful launches' instantiation, whose registers and schedule are then its own
 * (without the slot code: frame -0.8 %, chain -1.4 %, 1/8 share -2 %, profiles/r06_w_ab_defer_specialisation.log).
 * Counting launches always take GENERAL.  HITS: the fast instantiation of scenes whose bounces often hit again (the
 * upload's bounce_hit_share above kWgsHitShare, e.g. C3 fsuzane), with the later bounces' one-pass cull and pair build
 * (chain_trace_pairs); the other scenes' instantiation does not carry that code. */
template <bool MULTI, bool COUNT, bool HITS, bool GENERAL>
__global__ __launch_bounds__(kChainBlock) __attribute__((amdgpu_waves_per_eu(RTC_CHAIN_WAVES))) void rtc_render_chain(
    RenderParams P)
{
    if (RTC_CHAIN_PRIO > 0)
        __builtin_amdgcn_s_setprio(RTC_CHAIN_PRIO);
    DSECT_BEGIN(dtot);
    DMARK_INIT(dcur);
#ifdef RTC_DIAG
    const unsigned long long dWaveT0 = __builtin_amdgcn_s_memrealtime();
    unsigned dWaveItems = 0;
    unsigned long long dItemEnd[5] = {0, 0, 0, 0, 0};
#endif
    extern __shared__ __attribute__((aligned(64))) unsigned char sDyn[];
    __shared__ PowTablesLds sPow;
    __shared__ ChainWaveLds sWave[kChainBlock / 64];
    __shared__ int sWork; /* the workgroup's next item (see below) */
    __shared__ DevCluster sCl[kChunkClusters]; /* single-chunk scenes: the clusters, for the dense culls */
    if (!MULTI && threadIdx.x < P.clusterCount && threadIdx.x < kChunkClusters)
        sCl[threadIdx.x] = P.clusters[threadIdx.x];
    if (threadIdx.x == 0)
        sWork = 0;
    sPow.fill(threadIdx.x);
    const ChainStage S = chain_stage<MULTI>(P, sDyn);
    const float4 *sRec = S.rec;
    /* the staged primary filter records: always the LDS address (never null), used when P.chainPrimF */
    const DevPrimF *sPF = (const DevPrimF *)(sDyn + (MULTI ? 0 : (size_t)soa_slots(P.clusterCount * kClusterSize) * sizeof(DevTri)));
    const bool pfStaged = !GENERAL || P.chainPrimF != 0; /* (the fast instantiation runs only with the records staged) */
#ifdef RTC_DIAG
    if ((threadIdx.x & 63) < kDiagSects)
        s_rtc_sect[threadIdx.x >> 6][threadIdx.x & 63] = 0;
    static_assert(kChainBlock / 64 <= 4, "s_rtc_sect holds four waves");
#endif
    __syncthreads();
    sPow.attach(P.env);
    const int lane = threadIdx.x & 63;
    ChainWaveLds &W = sWave[threadIdx.x >> 6];
    const RngJump laneJump = rng_jump_by(7u * (unsigned)lane); /* s -> the state 7 lane draws later */
    /* the geometry pixels: kGeoLists sub-lists from rtc_tile_cull, taken as one concatenated index space
     * (l: the sub-list of item `it`, base: its first item).  Workgroup b owns the items b + k * gridDim.x; its
     * waves take the next k from an LDS counter, so a wave that drew cheap pixels takes more of them (a global
     * counter would serialise ~80 k same-address atomics across the XCDs; per-XCD returning counters, round 3,
     * shortened the kernel 4 % but made every workgroup retire at its end, so the sky pass no longer filled the
     * tail: frame 0.396 -> 0.42 ms). */
    int nextIt = 0;
    /* (Global item counters instead, round 5: the kernel 6 % shorter, the frame 3-4 % longer -- the sky pass no longer
     * fills its tail -- and small shares 17-28 % longer.  Items grouped by XCD, round 6 -- XCD group b % 8 taking the
     * (b % 8)-th eighth of the list, so that a tile's neighbouring pixels share an L2: frame 0.333 -> 0.358 ms, 1/8 share
     * 0.068 -> 0.079 ms, profiles/r06_c_ab_xcd_items_readlane_cull.log.) */
    /* (Runs of G / 8 consecutive items per XCD in every round of G = gridDim.x items, round 6 -- a tile's pixels under
     * one L2, so that their Color bytes merge before write-back: 1080p 1/4 and 1/8 shares 2-3 % longer, fsuzane +1 %,
     * profiles/r06_i_ab_cull_trim_xcd_runs_prefetch.log.) */
    const auto next_item = [&]() { return (int)blockIdx.x + atomicAdd(&sWork, 1) * (int)gridDim.x; };
    if (lane == 0)
        nextIt = next_item();
    /* (the launch constants below that are used once per item, window or escaped bounce are re-read from the kernarg
     * segment where they are used: KARG) */
#ifdef RTC_DIAG_COUNT /* diagnostic variant: the test counters on in every launch (rtc_diag_itemlog's tests) */
    constexpr bool counting = true;
#else
    constexpr bool counting = COUNT;
#endif
    unsigned segCalls = 0, segTraced = 0, segClusters = 0;
    unsigned long long segTests = 0, segSpec = 0;
#ifdef RTC_DIAG
    unsigned long long dIters = 0, dAlive = 0, dAct = 0, dWindows = 0, dUsed = 0, dIters2 = 0, dAlive2 = 0;
#endif
    /* the sub-lists' inclusive prefix counts, lane l < kGeoLists holding sub-list l's, loaded once per wave: an
     * item's sub-list is then a ballot, not a chain of dependent count loads as a wave's items pass the sub-lists */
    int incl = lane < kGeoLists ? min(P.geoCount[lane * kGeoCountStride], P.geoCap) : 0;
#pragma unroll
    for (int d = 1; d < kGeoLists; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d)
            incl += v;
    }
    const int nItems = __builtin_amdgcn_readlane(incl, kGeoLists - 1);
    /* Prefetch (round 5): an item's list entry and its tile's first two mask words were written by the tile cull on
     * other XCDs, so their first reads miss this XCD's L2; read as scalar loads at the item's start they were a chain
     * of dependent misses on the critical path of every item (round-4 stamps: item setup 17 % of the waves' lifetime).
     * Here they are VECTOR loads issued one item ahead: the next item's entry at this item's start, its tile's mask
     * dwords (lane j < 4: dword j) at this item's first bounce iteration, once the entry is back.  Vector loads return in
     * order and are waited for by vmcnt, so a scalar wait never completes them early.  Each lives in one register that
     * is consumed before it is reloaded (a loop-carried copy of an in-flight load would wait for it at the copy), and
     * neither is in flight at a loop preheader that flushes vmcnt (after the bounce loop, the walk's did). */
    const auto entry_of = [&](int it2) -> size_t {
        const int l = (int)__popcll(__ballot(lane < kGeoLists && incl <= it2));
        const int base = l ? __builtin_amdgcn_readlane(incl, l - 1) : 0;
        return (size_t)l * KARG(geoCap) + (size_t)(it2 - base);
    };
    const auto mask_dwords = [&](int code2) -> unsigned {
        const unsigned *mw = (const unsigned *)(KARG(tileMask) + (size_t)(code2 >> 6) * P.maskWords);
        return lane < 2 * P.maskWords && lane < 4 ? gload(mw, (size_t)lane) : 0u;
    };
    int it = __builtin_amdgcn_readfirstlane(nextIt);
    unsigned vc = 0, vm = 0; /* the current item's entry and mask dwords (vector registers) */
    if (it < nItems) {
        vc = gload(KARG(geoList), entry_of(it) + (size_t)vzero());
        vm = mask_dwords(__builtin_amdgcn_readfirstlane((int)vc));
    }
    if (lane == 0)
        nextIt = next_item();
    DMARK(dcur, 19); /* prologue: staging, tables, the first item */
    for (;;) {
        if (it >= nItems)
            break;
#ifdef RTC_DIAG
        const unsigned long long dItemT0 = __builtin_amdgcn_s_memrealtime();
        unsigned dItemWindows = 0;
        const unsigned long long dItemIters0 = dIters;
        const unsigned dBm0 = __atomic_load_n(&g_rtc_bmfall[(blockIdx.x * (kChainBlock / 64) + (threadIdx.x >> 6)) & 65535u],
                                              __ATOMIC_RELAXED);
        const unsigned long long dSect = lane < kItemSects ? s_rtc_sect[threadIdx.x >> 6][item_sect_id(lane)] : 0ull;
        unsigned long long dItemTests = 0;
#endif
        const int code = __builtin_amdgcn_readfirstlane((int)vc);
        const unsigned long long m0 = (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)vm, 0) |
                                      (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)vm, 1) << 32;
        const unsigned long long m1 = (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)vm, 2) |
                                      (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)vm, 3) << 32;
        /* the next item: its number (the LDS counter read at this item's previous start), its entry, and the counter for
         * the one after */
        const int itNext = __builtin_amdgcn_readfirstlane(nextIt);
        if (itNext < nItems)
            vc = gload(KARG(geoList), entry_of(itNext) + (size_t)vzero());
        /* the next item's mask dwords requested (none needed past the end) */
        bool maskNext = itNext >= nItems;
        if (lane == 0)
            nextIt = next_item();
        const int tile = code >> 6, bit = code & 63;
        const int tilesX = KARG(blocksX) * 2;
        const int x = (tile % tilesX) * 8 + (bit & 7), r = (tile / tilesX) * 8 + (bit >> 3);
        const int sh = KARG(rowBandShift); /* launch_row_y */
        const int y = KARG(rowStart) + ((r >> sh) * KARG(rowStride) << sh) + (r & ((1 << sh) - 1));
        V3 pdir; /* main.c:88-94, as primary_dir */
        {
            const int W = KARG(width), H = KARG(height);
            const float dx = (float)(x - W / 2) / (float)(H / 2);
            const float dy = (float)(y - H / 2) / (float)(H / 2);
            pdir = normalized(add(add(mul(KARG(ex), dx), mul(KARG(ey), dy)), mul(KARG(ez), KARG(fov))));
        }
        const unsigned long long *mask = KARG(tileMask) + (size_t)tile * P.maskWords;
        unsigned L = 0;
        if (counting)
            for (int w = 0; w < P.maskWords; ++w)
                L += (unsigned)__popcll(mask[w]);
        const unsigned seed = (unsigned)(x + y * KARG(width)); /* main.c:95 */
        const bool deferred = GENERAL && it < P.sampleCap; /* wave-uniform */
        Closest prim{999999.f, -1};
        if (GENERAL && P.hoist && P.spp > 0 && P.maxBounce > 0) {
            closest_primary_listed_lds(P, pdir, prim, mask, m0, m1, sPF, pfStaged);
            if (counting && lane == 0) {
                segTraced++;
                segTests += L;
            }
        }
        DMARK(dcur, 15); /* item setup */
        /* in-kernel sums (items without a deferred slot): the pixel's accumulator (main.c:97), component c in lane c */
        float acc = 0.f;
        int k = 0;       /* samples accumulated */
        unsigned jn = 0; /* state index (in units of 7 draws) of sample k */
        while (k < P.spp && P.maxBounce > 0) {
            /* window: the state indices the remaining samples likely span (the pixel's hits per sample so far, a
             * margin; the first window assumes one hit per sample) */
            const int need = P.spp - k;
            const int est = k > 0 ? (int)(((unsigned long long)need * jn + (unsigned)k - 1u) / (unsigned)k) : need;
            const int nAct = min(64, est + (est >> 3) + 1);
            const bool act = lane < nAct;
            /* the lane's start state: the seed advanced by 7 (jn + lane) draws = the wave-uniform state at jn,
             * then this lane's fixed jump by 7 lane draws (both affine LCG compositions, rng_advance) */
            const unsigned s0 = (unsigned)__builtin_amdgcn_readfirstlane((int)rng_advance(seed, 7u * jn));
            unsigned rng = s0 * laneJump.a + laneJump.c;
            DMARK(dcur, 0); /* window setup */
            /* ---- S_{jn + lane}: one calcColor (raytracing.c:262-296) ---- */
            V3 pos = KARG(origin), dir = pdir, rayColor{1.f, 1.f, 1.f}, light{0.f, 0.f, 0.f};
            int bounce = 0;
            unsigned hits = 0, calls = 0, tests = 0, clTests = 0;
            bool alive = act;
            for (int iter = 0; __any(alive); ++iter) {
                const bool first = iter == 0, bounce1 = iter == 1; /* wave-uniform */
#ifdef RTC_DIAG
                dIters++;
                dAlive += (unsigned long long)__popcll(__ballot(alive));
                if (iter >= 2) {
                    dIters2++;
                    dAlive2 += (unsigned long long)__popcll(__ballot(alive));
                }
#endif
                Closest c{999999.f, -1};
                if (first) { /* every live lane: the pixel's primary ray (bounce 0) */
                    if (alive) {
                        if (GENERAL && P.hoist) {
                            c = prim;
                        } else {
                            closest_primary_listed_lds(P, dir, c, mask, m0, m1, sPF, pfStaged);
                            if (counting)
                                tests += L;
                        }
                    }
                    DMARK(dcur, 1); /* primary trace */
                } else { /* bounce segments of the live lanes (the whole wave takes part) */
                    if (!maskNext) { /* the next item's mask dwords (see the prefetch above) */
                        vm = mask_dwords(__builtin_amdgcn_readfirstlane((int)vc));
                        maskNext = true;
                    }
                    unsigned t = 0;
                    c = chain_trace_pairs<MULTI, COUNT, HITS>(P, alive, bounce1, pos, dir, sRec, W, lane, t, sCl);
                    if (counting && alive) {
                        tests += t;
                        clTests += (unsigned)P.clusterCount;
                    }
                    DMARK(dcur, bounce1 ? 17 : 20); /* bounce trace: the first bounce (17), later ones (20); 14 table, 3
                                                     * cull, 4 pair build, 5 pair passes inside */
                }
                /* the state advance of this iteration's hits (7 draws per earlier hit), for lanes past the draw table */
                RngJump J{1u, 0u};
                if (!first && __ballot(alive && c.idx >= 0 && lane + iter >= nAct))
                    J = rng_jump_by(7u * (unsigned)iter); /* wave-uniform */
                if (alive) {
                    if (counting)
                        calls++;
                    bool endSample;
                    if (c.idx >= 0) {
                        DSECT_BEGIN(dc2);
                        hits++;
                        /* calcColor hit branch, raytracing.c:272-287 */
                        const V3 hitPoint = add(pos, mul(dir, c.dst)); /* raytracing.c:238 */
                        DevTri T;
                        DevMat M;
                        if (first) { /* the pixel's primary hit: the same triangle in every lane */
                            const int u = __builtin_amdgcn_readfirstlane(c.idx);
                            T = KLOAD(KARG(tris), u);
                            M = KLOAD(KARG(mats), u);
                        } else {
                            T = P.tris[c.idx]; /* (kernel-argument pointers: global loads, not flat) */
                            M = P.mats[c.idx];
                        }
                        const V3 normal{T.nx, T.ny, T.nz}, color{M.r, M.g, M.b};
                        /* the hit draws (see ChainWaveLds::draw): the primary hit computes the lane's own and enters
                         * them in the table (every active lane hits there: one primary ray per wave); a later hit
                         * reads entry lane + iter, or computes it when that is past the window's active lanes */
                        float4 D;
                        if (first || lane + iter >= nAct) {
                            unsigned s = first ? rng : rng * J.a + J.c;
                            const V3 rd = random_direction(s);
                            D = make_float4(rd.x, rd.y, rd.z, random_value(s));
                            if (first)
                                W.draw[lane] = D; /* read in later iterations, after chain_trace_pairs' LDS syncs */
                        } else {
                            D = W.draw[lane + iter];
                        }
                        const V3 diffuseDir = normalized(add(normal, V3{D.x, D.y, D.z}));
                        const V3 specularDir = reflect(dir, normal);
                        dir = lerp(diffuseDir, specularDir, M.smoothness);
                        pos = hitPoint;
                        const V3 emitted = mul(color, M.emission);
                        light = add(light, mulv(emitted, rayColor));
                        rayColor = mulv(rayColor, color);
                        const float p = fmax_ref(fmax_ref(rayColor.x, rayColor.y), rayColor.z);
                        endSample = p < D.w;
                        if (!endSample) {
                            rayColor = mul(rayColor, rcp_cr(p)); /* (float)(1.0 / p) */
                            bounce++;
                            endSample = bounce >= P.maxBounce;
                        }
                        DSECT_END(dc2, 2);
                    } else {
                        DSECT_BEGIN(dc6);
                        EnvParams env = KARG(env); /* the launch's sky and sun, the powf tables in LDS */
                        sPow.attach(env);
                        light = add(light, mulv(environment(dir, env), rayColor)); /* raytracing.c:291 */
                        endSample = true;
                        DSECT_END(dc6, 6);
                    }
                    if (endSample)
                        alive = false;
                }
                DMARK(dcur, iter < 2 ? 16 : 21); /* shading (2 hit, 6 environment inside); 21: after later bounces */
            }
            (void)bounce;
            /* ---- walk the chain through the window, accumulating in sample order (main.c:99) ---- */
            const V3 t = mul(light, KARG(invSpp)); /* calcColor(...) * (float)(1./spp), main.c:99 */
            const unsigned long long ones = __ballot(act && hits == 1u);
            unsigned mult = 0; /* how many accumulated samples this lane's S_j is */
            int p = 0;
            SampleSlot *slot = P.sampleBuf + (size_t)it * (size_t)P.spp;
            /* in-kernel sums: the window's samples are staged in sample order in LDS -- the pair list's space, free
             * until the next window's bounces; component c of staged sample i at stage[3 i + c] -- and lane c then adds
             * them in order.  Interleaved, the three summing lanes read three consecutive dwords (three banks) and the
             * staging lanes write at a stride of 3 dwords (a permutation of the 64 banks): no bank conflicts (round 4's
             * stage[64 c + i] put the three readers on one bank: 6.3 M conflict cycles per 1080p launch) */
            float *const stage = (float *)W.pair;
            int staged = 0;
            auto flush = [&]() {
                wave_lds_sync();
                if (lane < 3) {
                    const float *src = stage + lane;
#pragma unroll 8
                    for (int i = 0; i < staged; ++i)
                        acc = acc + src[3 * i];
                }
                wave_lds_sync();
                staged = 0;
            };
            while (k < P.spp && p < nAct) {
                const unsigned long long win = (nAct >= 64 ? ~0ull : ((1ull << nAct) - 1ull)) & (~0ull << p);
                const unsigned long long notOne = ~ones & win;
                const int q = notOne ? __builtin_ctzll(notOne) : nAct;
                const int take = min(q - p, P.spp - k);
                /* a run of one-hit samples: j advances by 1 */
                if (deferred) {
#ifndef RTC_AB_NO_SLOTS /* timing experiment only (the deferred slots' cost): nothing stored, no sum pass */
                    if (lane >= p && lane < p + take)
                        slot[k + lane - p] = SampleSlot{t.x, t.y, t.z};
#endif
                } else {
                    if (lane >= p && lane < p + take) {
                        const int i = 3 * (staged + lane - p);
                        stage[i] = t.x;
                        stage[i + 1] = t.y;
                        stage[i + 2] = t.z;
                    }
                    staged += take;
                }
                mult += (lane >= p && lane < p + take) ? 1u : 0u;
                k += take;
                p += take;
                if (k >= P.spp || p != q || q >= nAct)
                    break;
                /* lane q: a sample with h != 1 (two or more hits, or none when the primary ray misses) */
                const int hq = __builtin_amdgcn_readlane((int)hits, q);
                const float qx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.x), q));
                const float qy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.y), q));
                const float qz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t.z), q));
                const int m = hq == 0 ? P.spp - k : 1; /* a primary miss: every remaining sample is this one */
                if (deferred) {
                    for (int kk = k + lane; kk < k + m; kk += 64)
                        slot[kk] = SampleSlot{qx, qy, qz};
                } else if (m == 1) {
                    if (lane == q) {
                        stage[3 * staged] = t.x;
                        stage[3 * staged + 1] = t.y;
                        stage[3 * staged + 2] = t.z;
                    }
                    ++staged;
                } else { /* the staged samples first, then this one m times */
                    flush();
                    const float v = lane == 0 ? qx : (lane == 1 ? qy : qz);
                    for (int b = 0; b < m; ++b)
                        acc = acc + v;
                }
                mult += lane == q ? (unsigned)m : 0u;
                k += m;
                if (hq == 0)
                    break;
                p = q + hq;
            }
            if (!deferred)
                flush();
            jn += (unsigned)p;
#ifdef RTC_DIAG
            {
                unsigned long long tw = act ? tests : 0u;
                for (int o = 32; o > 0; o >>= 1)
                    tw += __shfl_xor(tw, o);
                dItemTests += tw;
            }
            dItemWindows++;
            dWindows++;
            dAct += (unsigned)nAct;
            dUsed += (unsigned long long)__popcll(__ballot(mult > 0));
#endif
            /* counters: committed samples (with multiplicity) and the tests of the discarded ones */
            if (counting) {
                segCalls += mult * calls;
                segTraced += mult * (P.hoist ? calls - 1u : calls);
                segTests += (unsigned long long)mult * tests;
                segClusters += mult * clTests;
                if (act && mult == 0)
                    segSpec += tests;
            }
            DMARK(dcur, 7); /* walk and sums */
        }
        if (deferred) {
            if (lane == 0)
                P.itemPix[it] = r * KARG(width) + x;
        } else if (P.geoColor) { /* merged sky pass: the pixel's three bytes as one word of its item */
            const unsigned b = float_to_u8(acc);
            const unsigned w = (unsigned)__builtin_amdgcn_readlane((int)b, 0) |
                               (unsigned)__builtin_amdgcn_readlane((int)b, 1) << 8 |
                               (unsigned)__builtin_amdgcn_readlane((int)b, 2) << 16;
            if (lane == 0)
                P.geoColor[it] = w;
            if (lane < 3 && P.accum)
                P.accum[3 * ((size_t)r * (size_t)KARG(width) + (size_t)x) + (size_t)lane] = acc;
        } else if (lane < 3) {
            const size_t o = 3 * ((size_t)r * (size_t)KARG(width) + (size_t)x) + (size_t)lane;
            P.colors[o] = float_to_u8(acc);
            if (P.accum)
                P.accum[o] = acc;
        }
        if (!maskNext) /* (an item without a bounce iteration) */
            vm = mask_dwords(__builtin_amdgcn_readfirstlane((int)vc));
#ifdef RTC_DIAG
        if (lane == 0 && it < kItemLog) {
            g_rtc_itemlog[it][0] = dItemT0;
            g_rtc_itemlog[it][1] = __builtin_amdgcn_s_memrealtime();
            g_rtc_itemlog[it][2] = (unsigned long long)dItemWindows |
                                   (unsigned long long)(__popcll(m0) + __popcll(m1)) << 16 |
                                   (unsigned long long)(blockIdx.x * (kChainBlock / 64) + (threadIdx.x >> 6)) << 32;
            const unsigned dBm1 = __atomic_load_n(
                &g_rtc_bmfall[(blockIdx.x * (kChainBlock / 64) + (threadIdx.x >> 6)) & 65535u], __ATOMIC_RELAXED);
            g_rtc_itemlog[it][3] = (dIters - dItemIters0) | (unsigned long long)(dBm1 - dBm0) << 16 | dItemTests << 32;
        }
        if (it < kItemSectLog && lane < kItemSects)
            g_rtc_itemsect[it][lane] = (unsigned)(s_rtc_sect[threadIdx.x >> 6][item_sect_id(lane)] - dSect);
#endif
        it = itNext;
#ifdef RTC_DIAG
        if (dWaveItems < 5)
            dItemEnd[dWaveItems] = __builtin_amdgcn_s_memrealtime();
        dWaveItems++;
#endif
        DMARK(dcur, 18); /* item tail: the pixel's colour */
    }
    DMARK(dcur, 15);
#ifdef RTC_DIAG
    DSECT_END(dtot, 13);
    {
        /* per-slot plain stores (see g_rtc_sectw): lanes 0..7, 13..21 the sections, 8..12 and 22, 23 the window statistics */
        const unsigned slotW = (blockIdx.x * (kChainBlock / 64) + (threadIdx.x >> 6)) % (unsigned)kWaveLog;
        unsigned long long v = lane < kDiagSects ? s_rtc_sect[threadIdx.x >> 6][lane] : 0ull;
        v = lane == 8 ? dIters : lane == 9 ? dAlive : lane == 10 ? dAct : lane == 11 ? dWindows : lane == 12 ? dUsed : v;
        v = lane == 22 ? dIters2 : lane == 23 ? dAlive2 : v;
        if (lane < kDiagSects)
            g_rtc_sectw[slotW][lane] = v;
    }
#endif
    if (counting)
        flush_counters(P, segCalls, segTraced, segTests, lane, segClusters, segSpec);
#ifdef RTC_DIAG
    if (lane == 0) {
        const unsigned w = (blockIdx.x * (kChainBlock / 64) + (threadIdx.x >> 6)) % (unsigned)kWaveLog;
        g_rtc_wavelog[w][0] = dWaveT0;
        g_rtc_wavelog[w][1] = __builtin_amdgcn_s_memrealtime();
        g_rtc_wavelog[w][2] = dWaveItems;
        for (int q = 0; q < 5; ++q)
            g_rtc_wavelog[w][3 + q] = dItemEnd[q];
    }
#endif
}

/* A kernel launch whose completion also records `stop` (null: a plain launch): the event is the dispatch's own
 * completion signal, so the stream gets no separate marker packet -- each marker on the launch stream cost ~5-7 us
 * before the next kernel (round 3: a hipEventRecord after the launch) */
template <typename... K, typename... A>
static hipError_t launch_stop(void (*k)(K...), dim3 g, dim3 b, size_t sh, hipStream_t st, hipEvent_t stop, A... args)
{
    if (stop) {
        hipExtLaunchKernelGGL(k, g, b, (std::uint32_t)sh, st, nullptr, stop, 0u, args...);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k, g, b, sh, st, args...);
    return hipGetLastError();
}

/* what an unjoined sky pass writes (rtcplan::Key): its buffers and everything that decides their values */
static rtcplan::Key sky_key(const RenderParams &P)
{
    rtcplan::Key k;
    memset(&k, 0, sizeof k);
    k.colors = (uint64_t)(uintptr_t)P.colors;
    k.accum = (uint64_t)(uintptr_t)P.accum;
    const V3 c[4] = {P.origin, P.ex, P.ey, P.ez}, e[4] = {P.env.sun, P.env.horizon, P.env.zenith, P.env.ground};
    for (int i = 0; i < 4; ++i) {
        k.cam[3 * i] = c[i].x, k.cam[3 * i + 1] = c[i].y, k.cam[3 * i + 2] = c[i].z;
        k.env[3 * i] = e[i].x, k.env[3 * i + 1] = e[i].y, k.env[3 * i + 2] = e[i].z;
    }
    k.cam[12] = P.fov;
    k.env[12] = P.env.focus;
    k.env[13] = P.env.intensity;
    const int dims[9] = {P.width, P.height, P.rows, P.rowStart, P.rowStride, P.spp, P.maxBounce, P.hoist, P.rowBandShift};
    memcpy(k.dims, dims, sizeof dims);
    return k;
}

static EnvParams env_of(const Scene &s)
{
    EnvParams e{};
    e.sun = V3{s.normalizedSunDirection.x, s.normalizedSunDirection.y, s.normalizedSunDirection.z};
    e.horizon = V3{s.skyColorHorizon.x, s.skyColorHorizon.y, s.skyColorHorizon.z};
    e.zenith = V3{s.skyColorZenith.x, s.skyColorZenith.y, s.skyColorZenith.z};
    e.ground = V3{s.groundColor.x, s.groundColor.y, s.groundColor.z};
    e.focus = s.sunFocus;
    e.intensity = s.sunIntensity;
    e.sunSkip = env_sun_skippable(e.focus, e.intensity);
    const float col[9] = {e.ground.x, e.ground.y, e.ground.z, e.horizon.x, e.horizon.y, e.horizon.z,
                          e.zenith.x, e.zenith.y, e.zenith.z};
    e.vanishLim = RTC_SUN_VANISH && e.sunSkip ? env_vanish_limit(e.focus, e.intensity, col) : -INFINITY;
    return e;
}


#ifdef RTC_AB_NO_SLOTS
constexpr bool kAbNoSlots = true; /* timing experiment only (RTC_EXPERIMENT): deferred samples neither stored nor summed */
#else
constexpr bool kAbNoSlots = false;
#endif
extern "C" int rtc_render_rows_async(const RtcDeviceScene *s, const Scene *scene, const RtcCamera *cam,
                                     const RtcRenderDesc *d, void *dColors, float *dAccum,
                                     unsigned long long *dSegments, void *stream)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "rtc_render_rows_async: null scene");
    RtcDeviceScene *const ms = const_cast<RtcDeviceScene *>(s);
    /* The hooks are one-shot: this launch takes the events armed before it and forgets them -- before any early
     * return, so a later launch never records an event its caller has since released (rtc_scene_set_geometry_event /
     * _frame_event); a launch that fails records neither */
    const hipEvent_t geoEvent = s->geoEvent, frameEvent = s->frameEvent;
    ms->geoEvent = nullptr;
    ms->frameEvent = nullptr;
    if (!scene || !cam || !d || !dColors)
        return rtc_fail(RTC_EINVAL, "rtc_render_rows_async: null argument");
    if (d->width <= 0 || d->height <= 0 || d->rowStride <= 0 || d->rowStart < 0 || d->rowBand < 0 || d->rowBand > 64 ||
        (d->rowBand & (d->rowBand - 1)) != 0)
        return rtc_fail(RTC_EINVAL, "rtc_render_rows_async: bad geometry %dx%d rows %d+k*%d", d->width, d->height,
                        d->rowStart, d->rowStride);
    if ((long long)d->width * d->height > (1ll << 31) / 4)
        return rtc_fail(RTC_EINVAL, "frame too large");
    if (d->flags & (RTC_F_COOP4 | RTC_F_COOP8 | RTC_F_PIPE | RTC_F_SPEC))
        return rtc_fail(RTC_EINVAL, "rtc_render_rows_async: RTC_F_COOP4 / COOP8 / PIPE / SPEC name kernels that were "
                                    "removed (rtc_render_chain renders every geometry pixel)");
    const int rows = rtc_rows_selected(d);
    /* the scene's buffers, scratch and kernels live on s->device; the caller's current device is restored */
    RtcDeviceGuard guard(s->device);
    if (!guard.ok())
        return rtc_fail(RTC_ENODEV, "rtc_render_rows_async: cannot select the scene's device %d", s->device);
    if (rows == 0) { /* nothing to render: the (empty) frame is complete once `stream` gets here */
        for (hipEvent_t ev : {geoEvent, frameEvent})
            if (ev)
                HIP_TRY(hipEventRecord(ev, (hipStream_t)stream));
        return 0;
    }
    RenderParams P;
    memset(&P, 0, sizeof P);
    P.tris = s->tris;
    P.mats = s->mats;
    P.spheres = s->spheres;
    P.colors = (unsigned char *)dColors;
    P.accum = dAccum;
    P.segments = dSegments;
    P.segSlots = s->segSlots;
    P.triCount = s->triCount;
    P.triPadded = s->triPadded;
    P.clTris = s->clTris;
    P.clusters = s->clusters;
    P.chunks = s->chunks;
    P.chunkCount = s->chunkCount;
    P.clusterCount = s->clusterCount;
    P.clusterCull = !(d->flags & RTC_F_NO_CLUSTER_CULL);
    P.sphereCount = d->trianglesOnly ? 0 : s->sphereCount;
    P.maskWords = s->maskWords;
    P.width = d->width;
    P.height = d->height;
    P.rows = rows;
    P.rowStart = d->rowStart;
    P.rowStride = d->rowStride;
    P.rowBandShift = d->rowBand > 1 ? __builtin_ctz((unsigned)d->rowBand) : 0;
    P.spp = d->spp;
    P.maxBounce = d->maxBounce;
    P.hoist = (d->flags & RTC_F_HOIST_PRIMARY) ? 1 : 0;
    P.invSpp = d->spp > 0 ? (float)(1. / (double)d->spp) : 0.f;
    P.origin = v3(cam->origin);
    P.ex = v3(cam->ex);
    P.ey = v3(cam->ey);
    P.ez = v3(cam->ez);
    P.fov = cam->fov;
    P.env = env_of(*scene);
    hipStream_t st = (hipStream_t)stream;
    /* every ordering decision -- slot, streams, events, which kernels -- comes from the planner (rtc_plan.h); this
     * function executes its operations */
    rtcplan::Request rq{};
    rq.stream = (uint64_t)(uintptr_t)st;
    rq.flags = d->flags;
    rq.width = d->width;
    rq.rows = rows;
    rq.rowStride = d->rowStride;
    rq.spp = d->spp;
    rq.sphereCount = P.sphereCount;
    rq.triPadded = s->triPadded;
    rq.maskWords = s->maskWords;
    rq.segments = dSegments != nullptr;
    rq.key = sky_key(P);
    memcpy(rq.origin, &P.origin, sizeof rq.origin);
    rq.noMerge = !RTC_SKY_MERGE;
    static thread_local rtcplan::Plan pl;
    rtcplan::plan_launch(s->plan, rq, pl);
    /* the saved state claims only what has been enqueued: until every operation below is, a later launch sees none of
     * this launch's primary records or counter zeroing (it re-runs rtc_prep_primary) */
    ms->plan.prepValid[pl.half] = false;
    ms->plan.cullValid = false;
    if (pl.needCst2) { /* created on first use: whole frames keep three streams (one more costs them ~1 %) */
        int leastPrio = 0, greatestPrio = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&leastPrio, &greatestPrio));
        HIP_TRY(hipStreamCreateWithPriority(&ms->cst2, hipStreamNonBlocking, greatestPrio));
        ms->plan.cst2 = true;
    }
    if (pl.scratchGrow) { /* every slot (hipFree synchronises the device: no launch still reads the old scratch) */
        if (ms->scratch)
            HIP_TRY(hipFree(ms->scratch));
        ms->scratch = nullptr;
        ms->plan.scratchCap = 0;
        HIP_TRY(hipMalloc(&ms->scratch, pl.scratchNeed));
        ms->plan.scratchCap = pl.scratchNeed;
    }
    if (pl.samplesGrow) {
        if (ms->samples)
            HIP_TRY(hipFree(ms->samples));
        ms->samples = nullptr;
        ms->plan.samplesCap = 0;
        HIP_TRY(hipMalloc(&ms->samples, pl.samplesNeed));
        ms->plan.samplesCap = pl.samplesNeed;
    }
    const int half = pl.half;
    P.primF = s->primF + (size_t)half * s->primStride;
    P.primX = s->primX + (size_t)half * s->primStride;
    P.blocksX = (int)pl.gridX;
    unsigned long long *mask = nullptr, *pixMask = nullptr, *superMask = nullptr;
    unsigned *weight = nullptr;
    int *order = nullptr;
    if (pl.cull) {
        unsigned char *slot = s->scratch + pl.slotOffset;
        mask = (unsigned long long *)(slot + pl.lay.mask);
        pixMask = (unsigned long long *)(slot + pl.lay.pixMask);
        weight = (unsigned *)(slot + pl.lay.weight);
        order = (int *)(slot + pl.lay.order);
        superMask = (unsigned long long *)(slot + pl.lay.superMask);
        if (pl.merge) {
            P.pixItem = (unsigned *)(slot + pl.lay.pixItem);
            P.geoColor = (unsigned *)(slot + pl.lay.geoColor);
        }
        P.tileMask = mask;
        P.pixMask = pixMask;
        if (!pl.fused)
            P.order = (d->flags & RTC_F_NO_REORDER) ? nullptr : order;
    }
    if (pl.superCull) {
        P.superMask = superMask;
        P.superX = (int)pl.superX;
    }
    if (pl.chain) {
        P.geoCount = s->geoCounts + (size_t)pl.geoSet * kGeoSetInts;
        P.geoCountNext = s->geoCounts + (size_t)pl.geoSetNext * kGeoSetInts;
        P.geoList = (int *)(s->scratch + pl.slotOffset + pl.lay.geoList);
        P.geoCap = pl.geoCap;
        P.cullPrio = pl.cullPrio;
        if (pl.sampleCap > 0) {
            P.sampleBuf = (SampleSlot *)s->samples;
            P.itemPix = (int *)(s->samples + (size_t)pl.sampleCap * (size_t)d->spp * sizeof(SampleSlot));
            P.sampleCap = pl.sampleCap;
        }
    }
    /* dynamic LDS of the geometry kernel: the clustered records (single-chunk scenes), then the primary filter records
     * when the block stays within its workgroups per CU */
    const int wgsPerCu = pl.smallShare ? RTC_CHAIN_WGS_SHARE : s->chainWgsFull;
    const size_t recLds = s->chunkCount <= 1 ? (size_t)soa_slots(s->clusterCount * kClusterSize) * sizeof(DevTri) : 0;
    const size_t pfLds = (size_t)s->triPadded * sizeof(DevPrimF);
    P.chainPrimF = s->chunkCount <= 1 && kChainStaticLds + recLds + pfLds <= kCuLds / (size_t)wgsPerCu;
    const size_t floorLds = chain_lds_floor(wgsPerCu);
    const size_t chainDyn = std::max<size_t>(recLds + (P.chainPrimF ? pfLds : 0),
                                             floorLds > kChainStaticLds ? floorLds - kChainStaticLds : 0);
    const dim3 grid(pl.gridX, pl.gridY);
    const hipStream_t streams[rtcplan::kStreams] = {st, s->cst, ms->cst2, s->side};
    const auto event = [&](int e) -> hipEvent_t {
        if (e >= rtcplan::kEvSkyDone0 && e < rtcplan::kEvSkyDone0 + kSkySlots)
            return s->evSkyDone[e - rtcplan::kEvSkyDone0];
        if (e >= rtcplan::kEvGeoDone0 && e < rtcplan::kEvGeoDone0 + kSkySlots)
            return s->evGeoDone[e - rtcplan::kEvGeoDone0];
        switch (e) {
        case rtcplan::kEvCullSync: return s->evCullSync;
        case rtcplan::kEvFork: return s->evFork;
        case rtcplan::kEvJoin: return s->evJoin;
        case rtcplan::kEvFrame: return frameEvent;
        case rtcplan::kEvGeometry: return geoEvent;
        default: return nullptr;
        }
    };
    for (int i = 0; i < pl.nOps; ++i) {
        const rtcplan::Op &op = pl.ops[i];
        const hipStream_t os = streams[op.stream];
        const hipEvent_t ev = event(op.event);
        if (op.kind == rtcplan::kOpRecord) {
            if (ev) /* (the caller's hooks may be unarmed) */
                HIP_TRY(hipEventRecord(ev, os));
            continue;
        }
        if (op.kind == rtcplan::kOpWait) {
            HIP_TRY(hipStreamWaitEvent(os, ev, 0));
            continue;
        }
        switch (op.kernel) {
        case rtcplan::kKPrep:
            hipLaunchKernelGGL(rtc_prep_primary, dim3((s->triPadded + 8 + 63) / 64), dim3(64), 0, os, s->tris,
                               const_cast<DevPrimF *>(P.primF), const_cast<DevPrimX *>(P.primX),
                               s->triPadded > 0 ? s->triPadded + 8 : 0, P.origin, pl.prepCounts ? P.geoCount : nullptr);
            HIP_TRY(hipGetLastError());
            break;
        case rtcplan::kKSuperCull:
            hipLaunchKernelGGL(rtc_super_cull, dim3(pl.superX, pl.superY), dim3(64), 0, os, P, superMask);
            HIP_TRY(hipGetLastError());
            break;
        case rtcplan::kKTileCull:
            HIP_TRY(launch_stop(rtc_tile_cull, grid, dim3(kBlock), (size_t)s->maskWords * sizeof(unsigned long long), os, ev,
                                P, mask, weight, pixMask));
            break;
        case rtcplan::kKSky: {
            if (s->timing)
                HIP_TRY(hipEventRecord(s->evSky0, os));
            const bool skyWide = pl.smallShare && (size_t)d->width * (size_t)rows > 400000; /* four-wave workgroups */
            const bool general = P.geoColor || P.hoist || P.accum || P.segments;
            const dim3 g4((d->width + 63) / 64, (rows + 3) / 4), g1((d->width + 63) / 64, rows);
            if (skyWide && general)
                hipLaunchKernelGGL((rtc_render_sky_rows<4, true>), g4, dim3(256), 0, os, P);
            else if (skyWide)
                hipLaunchKernelGGL((rtc_render_sky_rows<4, false>), g4, dim3(256), 0, os, P);
            else if (general)
                hipLaunchKernelGGL((rtc_render_sky_rows<1, true>), g1, dim3(64), 0, os, P);
            else
                hipLaunchKernelGGL((rtc_render_sky_rows<1, false>), g1, dim3(64), 0, os, P);
            HIP_TRY(hipGetLastError());
            if (s->timing)
                HIP_TRY(hipEventRecord(s->evSky1, os));
            break;
        }
        case rtcplan::kKChain: {
            if (s->timing)
                HIP_TRY(hipEventRecord(s->evHeavy0, os));
            const dim3 cg((unsigned)(wgsPerCu * s->cuCount)), cb(kChainBlock);
            const bool defer = P.sampleCap > 0 || P.hoist || !P.chainPrimF; /* (GENERAL) */
            const bool hits = s->chainWgsFull == RTC_CHAIN_WGS_HIT && RTC_CHAIN_WGS_HIT != RTC_CHAIN_WGS_FULL;
            if (s->chunkCount > 1 && dSegments)
                HIP_TRY(launch_stop(rtc_render_chain<true, true, false, true>, cg, cb, chainDyn, os, ev, P));
            else if (s->chunkCount > 1) /* (multi-chunk scenes never stage the primary records: GENERAL) */
                HIP_TRY(launch_stop(rtc_render_chain<true, false, false, true>, cg, cb, chainDyn, os, ev, P));
            else if (dSegments)
                HIP_TRY(launch_stop(rtc_render_chain<false, true, false, true>, cg, cb, chainDyn, os, ev, P));
            else if (defer)
                HIP_TRY(launch_stop(rtc_render_chain<false, false, false, true>, cg, cb, chainDyn, os, ev, P));
            else if (hits)
                HIP_TRY(launch_stop(rtc_render_chain<false, false, true, false>, cg, cb, chainDyn, os, ev, P));
            else
                HIP_TRY(launch_stop(rtc_render_chain<false, false, false, false>, cg, cb, chainDyn, os, ev, P));
            if (s->timing) /* the chain kernel alone (rocprof's rtc_render_chain row) */
                HIP_TRY(hipEventRecord(s->evHeavy1, os));
            break;
        }
        case rtcplan::kKAccum:
            if (!kAbNoSlots) {
                const unsigned g = (unsigned)std::min<size_t>(((size_t)P.sampleCap + 255) / 256, 1024);
                HIP_TRY(launch_stop(rtc_accumulate_samples, dim3(g), dim3(256), 0, os, ev, P));
            } else if (ev) {
                HIP_TRY(hipEventRecord(ev, os));
            }
            break;
        case rtcplan::kKOrder:
            hipLaunchKernelGGL(rtc_order_blocks, dim3(1), dim3(1024), 0, os, weight, (int)pl.blocks, order);
            HIP_TRY(hipGetLastError());
            break;
        case rtcplan::kKRender:
            if (P.sphereCount > 0 && pl.debug)
                hipLaunchKernelGGL((rtc_render_kernel<true, true>), grid, dim3(kBlock), 0, os, P);
            else if (P.sphereCount > 0)
                hipLaunchKernelGGL((rtc_render_kernel<true, false>), grid, dim3(kBlock), 0, os, P);
            else if (pl.debug)
                hipLaunchKernelGGL((rtc_render_kernel<false, true>), grid, dim3(kBlock), 0, os, P);
            else
                hipLaunchKernelGGL((rtc_render_kernel<false, false>), grid, dim3(kBlock), 0, os, P);
            HIP_TRY(hipGetLastError());
            break;
        case rtcplan::kKReduce:
            hipLaunchKernelGGL(rtc_reduce_segments, dim3(1), dim3(kSegSlots), 0, os, s->segSlots, dSegments);
            HIP_TRY(hipGetLastError());
            break;
        default:
            return rtc_fail(RTC_EINVAL, "rtc_render_rows_async: unknown planned kernel %d", op.kernel);
        }
    }
    ms->timed = pl.fused && s->timing;
    ms->plan = pl.after; /* every operation is enqueued */
    return 0;
}

/* ---- row de-interleave after a gather (bytes) ----------------------------------------------------- */
__global__ __launch_bounds__(256) void rtc_deinterleave_kernel(const unsigned char *__restrict__ in, int parts,
                                                                int rowsPerPart, int rowBytes, int height, int bandShift,
                                                                unsigned char *__restrict__ out)
{
    /* one block-row per output row y: band b = y / B of part b % parts, the part's band b / parts */
    const int y = blockIdx.y;
    if (y >= height)
        return;
    const int b = y >> bandShift, j = y & ((1 << bandShift) - 1);
    const int g = b % parts, k = ((b / parts) << bandShift) + j;
    const unsigned char *src = in + ((size_t)g * rowsPerPart + k) * (size_t)rowBytes;
    unsigned char *dst = out + (size_t)y * rowBytes;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rowBytes; i += gridDim.x * blockDim.x)
        dst[i] = src[i];
}

extern "C" int rtc_deinterleave_bands_async(const void *dCompact, int parts, int rowsPerPart, int width, int height,
                                            int rowBand, void *dOut, void *stream)
{
    if (!dCompact || !dOut || parts <= 0 || width <= 0 || height <= 0 || rowBand < 0 || rowBand > 64 ||
        (rowBand & (rowBand - 1)) != 0)
        return rtc_fail(RTC_EINVAL, "rtc_deinterleave_bands_async: bad argument");
    const int B = rowBand > 1 ? rowBand : 1;
    /* every part holds its bands' rows: part 0's count is the largest */
    RtcRenderDesc d0{};
    d0.width = width, d0.height = height, d0.rowStart = 0, d0.rowStride = parts, d0.rowBand = B;
    if (rowsPerPart < rtc_rows_selected(&d0))
        return rtc_fail(RTC_EINVAL, "rtc_deinterleave_bands_async: %d rows per part, part 0 has %d", rowsPerPart,
                        rtc_rows_selected(&d0));
    const int rowBytes = width * 3;
    dim3 grid((rowBytes + 255) / 256 < 8 ? (rowBytes + 255) / 256 : 8, height);
    hipLaunchKernelGGL(rtc_deinterleave_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char *)dCompact, parts, rowsPerPart, rowBytes, height, __builtin_ctz((unsigned)B),
                       (unsigned char *)dOut);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int rtc_deinterleave_async(const void *dCompact, int parts, int rowsPerPart, int width, int height,
                                      void *dOut, void *stream)
{
    if (!dCompact || !dOut || parts <= 0 || width <= 0 || height <= 0 || rowsPerPart * parts < height)
        return rtc_fail(RTC_EINVAL, "rtc_deinterleave_async: bad argument");
    return rtc_deinterleave_bands_async(dCompact, parts, rowsPerPart, width, height, 1, dOut, stream);
}

/* A frame copy with a small footprint (rtc_copy_async): `blocks` workgroups stream 16-byte words (the byte tail
 * by the first lanes), e.g. from HBM into pinned host memory over PCIe, so a D2H of Color[] occupies a few CU
 * slots instead of one workgroup on every CU (the runtime's blit kernel) while the render kernels run. */
__global__ __launch_bounds__(256) void rtc_copy_kernel(const unsigned char *__restrict__ src,
                                                       unsigned char *__restrict__ dst, size_t bytes)
{
    const size_t n16 = bytes / 16;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint4 *s16 = (const uint4 *)src;
    uint4 *d16 = (uint4 *)dst;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) { /* four independent 16-byte loads in flight per lane */
        const uint4 a = s16[i], b = s16[i + stride], c = s16[i + 2 * stride], d = s16[i + 3 * stride];
        d16[i] = a;
        d16[i + stride] = b;
        d16[i + 2 * stride] = c;
        d16[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride)
        d16[i] = s16[i];
    const size_t t = n16 * 16 + blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < bytes)
        dst[t] = src[t];
}

extern "C" int rtc_copy_async(void *dst, const void *src, size_t bytes, int blocks, void *stream)
{
    if ((!dst || !src) && bytes)
        return rtc_fail(RTC_EINVAL, "rtc_copy_async: null pointer");
    if (bytes == 0)
        return 0;
    if ((((size_t)dst | (size_t)src) & 15) != 0)
        return rtc_fail(RTC_EINVAL, "rtc_copy_async: pointers must be 16-byte aligned");
    if (blocks <= 0)
        blocks = 32;
    hipLaunchKernelGGL(rtc_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned char *)src, (unsigned char *)dst, bytes);
    HIP_TRY(hipGetLastError());
    return 0;
}

/*
 * rtc_layout.h -- the device scene as librtc.so's translation units share it: the HBM records the kernels read
 * (triangles with precomputed edges, materials, per-launch primary records, triangle clusters), the bounce-ray cluster
 * test, and the per-scene host state (RtcDeviceScene: buffers, streams, the launch-ordering state).
 * Reference layout it replaces: Triangle / Sphere / Material (raytracing.h:7-69) and the arrays main.c:229-243 builds.
 */
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/rtc.h"
#include "rtc_device.h"
#include "rtc_plan.h"

using namespace rtcdev;

/* ---- device scene layout ------------------------------------------------------------------------- */
/* 64 B per triangle, read wave-uniformly by s_load_dwordx16: A, AB, AC, N (the reference's stored normal). */
struct __attribute__((aligned(64))) DevTri {
    float ax, ay, az, abx, aby, abz, acx, acy, acz, nx, ny, nz, pad0, pad1, pad2, pad3;
};
/* material, read only for the winning triangle */
struct __attribute__((aligned(32))) DevMat {
    float r, g, b, emission, smoothness, pad0, pad1, pad2;
};
struct __attribute__((aligned(16))) DevSphere {
    float cx, cy, cz, radius, r, g, b, emission, smoothness, pad0, pad1, pad2;
};
/* Per-launch records for primary rays (bounce 0): every primary ray starts at the camera origin O, so all
 * the quantities rayTriangle derives from the ray are LINEAR in its direction d:
 *   nd = d.N,  det = AB.(d x AC) = d.Gd,  uu = s0.(d x AC) = d.Gu,  vv = d.q0
 * with s0 = O - A, q0 = s0 x AB, Gd = AC x AB, Gu = AC x s0 (raytracing.c:189-206).
 * DevPrimF drives an exact-safe FILTER: FMA dot products against these vectors plus per-triangle error
 * bounds (rtc_prep_primary derives them in double) reject a lane only when the reference's own float
 * arithmetic provably rejects it.  Surviving lanes run the reference arithmetic with DevPrimX (AB, AC, s0,
 * q0 and dot(AC, q0) computed once per launch with the reference's f32 ops: bit-exact).
 *
 * Orientation folding: a hit needs dst = dot(AC, q0) * invDet >= EPSILON > 0, so sign(det) must equal the
 * sign of dAC0 = dot(AC, q0) -- a per-triangle constant for primary rays.  The filter vectors are stored
 * pre-multiplied by sigma = sign(dAC0) (exact negation), which turns the per-lane sign normalisation into
 * nothing: a lane is a candidate iff  sigma*det~ >= c  and  min(sigma*u~, sigma*v~, sigma*w~) >= -m. */
struct __attribute__((aligned(64))) DevPrimF { /* 64 B: one s_load_dwordx16 */
    float nx, ny, nz, mnd;      /* N and the nd margin (-inf: the triangle can never be hit, skip it) */
    float gdx, gdy, gdz, c;     /* sigma*Gd and the det threshold c = EPSILON - ed, rounded down */
    float gux, guy, guz, negm;  /* sigma*Gu and -m (the combined edge margin, negated) */
    float q0x, q0y, q0z, pad0;  /* sigma*q0 */
};
struct __attribute__((aligned(64))) DevPrimX {
    float abx, aby, abz, acx, acy, acz, s0x, s0y, s0z, q0x, q0y, q0z, dac0, pad[3];
};

/* ---- triangle clusters for bounce rays (rtc_render_chain) -----------------------------------------------
 * The triangles are grouped into clusters of kClusterSize (spatial median splits, rtc_build_clusters); a
 * bounce ray skips a whole cluster when its half-line provably passes farther from the cluster's bounding
 * ball than any point rayTriangle could report.  Bound (SURVEY Appendix A arithmetic, unit roundoff
 * u = 2^-24): for a reported hit (|det| >= EPSILON, u, v in the triangle, dst >= EPSILON) the exact point
 * pos + dst*dir lies within
 *     eps = rho * (alpha + beta * S) + gamma * (S + E)
 * of the triangle, where rho >= |dir|, S >= |pos - A|, E = the cluster's longest AB / AC edge, and
 *     beta = F k 45 u E^2 / EPSILON,  alpha = F k 32 u E^3 / EPSILON,  k = 1 / (1 - 8 u E^2 rhoMax / EPSILON)
 * (forward error of the f32 cross / dot products over the Cramer solution, divided by |det| >= EPSILON;
 * safety factor F = 4; gamma covers the f32 evaluation of the cull test itself).  Clusters with
 * 8 u E^2 rhoMax / EPSILON >= 1/2, and rays with |dir|_1 > rhoMax, are never culled. */
constexpr int kClusterSize = 8;
constexpr int kChunkClusters = 32; /* clusters per chunk (one 32-bit cull mask per lane in rtc_render_chain) */
constexpr float kClusterRhoMax = 4.f;
constexpr float kClusterGamma = 2e-5f;
struct __attribute__((aligned(32))) DevCluster {
    float cx, cy, cz, r;          /* bounding ball (every vertex A, A+AB, A+AC of the cluster inside) */
    float alpha, beta, gammaE, e; /* the eps terms above: alpha, beta, gamma*E (or +inf: never cull), E */
};

/* The scene's own events only order its streams on one device (the caller's frame / geometry events keep their
 * flags): no system-scope fence when they are recorded (1/8 share 0.100 -> 0.094 ms, round 3) */
constexpr unsigned kOrderEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;
/* An unjoined sky pass (RTC_F_OVERLAP) writes its launch's Color (and accumulator) rows: what it writes where */
constexpr int kSkySlots = 8;
#ifndef RTC_CHAIN_WGS_FULL
#define RTC_CHAIN_WGS_FULL 3
#endif
/* Small shares of more pixels (the 1080p 1/4 share, 518 k px) run the tile cull at issue priority 3 as well: the next
 * share's cull then competes on equal terms with this share's geometry kernel (1/4 share 0.1205 -> 0.1170 ms; the 1/8
 * share measured no better that way, profiles/r05_cpq_ab_cull_priority.log) */
constexpr size_t kCullPrioMinPixels = 400000;
/* Wave priority of the geometry kernel (s_setprio): its waves are issued before the sky pass's on a shared SIMD.  A row
 * share's chain kernel runs ~3 pixels per wave; as its waves retire, sky waves fill their slots and the remaining chain
 * waves -- the share's critical path -- got a sixth of the issue: a wave's third and fourth pixels took 2-7x its first
 * (tools/wave_spread.py).  Round 5: 1080p 1/8 share 0.0757 -> 0.0697 ms, whole frames unchanged (the sky pass still
 * fills the chain kernel's idle slots); the tile cull at priority 3 too within noise of it
 * (profiles/r05_pr_ab_wave_priority.log) */
#ifndef RTC_CHAIN_PRIO
#define RTC_CHAIN_PRIO 3
#endif
#ifndef RTC_CHAIN_WGS_HIT
#define RTC_CHAIN_WGS_HIT 4 /* whole frames of scenes whose bounce-hit share (bounce_hit_share) exceeds kWgsHitShare */
#endif
constexpr double kWgsHitShare = 0.15;

/* rtc_render_chain's geometry-pixel sub-lists: kGeoLists counters, kGeoCountStride ints (one 128-B line) apart; a ring
 * of kGeoRing counter sets of kGeoSetInts ints (see RtcDeviceScene::geoCounts) */
constexpr int kGeoLists = 16, kGeoCountStride = 32;
constexpr int kGeoRing = 16, kGeoSetInts = kGeoLists * kGeoCountStride;
static_assert(kGeoSetInts >= kGeoLists * kGeoCountStride, "a counter set holds every sub-list counter");
static_assert(kSkySlots == rtcplan::kSlots && kGeoRing == rtcplan::kGeoRing && kGeoLists == rtcplan::kGeoLists &&
                  kGeoCountStride == rtcplan::kGeoCountStride,
              "the planner's slot and counter-set layout is the device's");
struct RtcDeviceScene {
    int device;
    int cuCount; /* compute units of the device (the persistent chain kernel's workgroups are a multiple of it) */
    int triCount, triPadded, sphereCount; /* triPadded: multiple of kUnroll, zero (never-hit) records */
    int clusterCount;   /* ceil(triCount / kClusterSize) */
    DevTri *clTris;     /* clusterCount * kClusterSize records in cluster order, pad0 = reference index (int) */
    DevCluster *clusters;
    DevCluster *chunks; /* chunkCount balls over kChunkClusters consecutive clusters */
    int chunkCount;
    DevTri *tris;
    DevMat *mats;
    DevSphere *spheres;
    /* per-launch primary records, one copy per scratch slot (primStride records each), written by rtc_prep_primary:
     * an overlapped launch's preparation (on the cull stream) may run while the previous frame's geometry kernel still
     * reads its own copy */
    DevPrimF *primF;
    DevPrimX *primX;
    size_t primStride;
    /* per-launch scratch (rtc_tile_cull / rtc_order_blocks): kSkySlots slots of the candidate bit-sets, pixel masks,
     * weights, dispatch order, geometry-pixel sub-lists and superblock survivors (rtcplan::Layout); grown on demand
     * (plan.scratchCap bytes) */
    unsigned char *scratch;
    /* rtc_render_chain's sub-list counters: a ring of kGeoRing sets, set q % kGeoRing for the q-th split launch;
     * each launch's tile cull zeroes the next launch's set */
    int *geoCounts;
    double hitShare;  /* bounce_hit_share at upload */
    int chainWgsFull; /* rtc_render_chain workgroups per CU for whole frames */
    /* every ordering decision's state: slots, pending sky passes, counter sets, prep records (rtc_plan.h) */
    rtcplan::State plan;
    /* streams: overlapped launches prepare, cull and run their geometry kernel on `cst` or `cst2` (high priority, by
     * slot parity); the sky pass runs on `side` (low priority) */
    hipStream_t cst;
    hipStream_t cst2; /* the second cull stream (odd slots; created on first use) */
    hipStream_t side;
    /* the scene's ordering events (rtcplan::Event): the caller stream's position when the culls move to a cull stream,
     * the tile cull's completion (the sky pass forks there), the sky pass's end, and per slot the end of its launch's
     * sky pass (after its geometry kernel) and of its geometry kernel */
    hipEvent_t evCullSync, evFork, evJoin;
    hipEvent_t evSkyDone[kSkySlots], evGeoDone[kSkySlots];
    hipEvent_t frameEvent; /* caller's (rtc_scene_set_frame_event) or null */
    /* caller's event (rtc_scene_set_geometry_event): recorded on the caller's stream once a launch's
     * geometry-pixel kernels are enqueued (before the join with the sky pass); null: none */
    hipEvent_t geoEvent;
    /* rtc_render_chain's deferred accumulation: the accumulated samples' radiance per geometry pixel (grown on demand,
     * <= kSampleBufBudget bytes: plan.samplesCap) */
    unsigned char *samples;
    int maskWords;     /* ceil(triPadded / 64) */
    unsigned long long *segSlots; /* per-launch partial segment counters */
    /* timing events around the split launch's two kernels (rtc_scene_kernel_times) */
    hipEvent_t evHeavy0, evHeavy1, evSky0, evSky1;
    bool timing; /* record them (rtc_scene_set_timing; off by default: each record costs the launch a few us) */
    bool timed;  /* the last launch was a split launch that recorded them */
};

/* True when the bounce ray (pos, dir) provably cannot hit any triangle of cluster K (see DevCluster): the
 * half-line's distance to the ball centre exceeds T >= r + eps.  rho = |dir|_1 >= |dir| bounds the eps terms;
 * dd = dir.dir.  With w = centre - pos and b = w.dir, the half-line's closest point to the centre is interior
 * when b > 0, at distance |w x dir| / |dir|, else the origin, at |w|.  |w x dir|^2 is evaluated by Lagrange's
 * identity w2 dd - b^2 (FMA dots, each within 3u relative; the cancellation is covered by an explicit margin of
 * 25u w2 dd >= the evaluation error) and compared with T^2 dd: the 1.00001 factor on T covers dd's own error.
 * The f32 evaluation of w, S and T is covered by the gamma terms (rtc_build_clusters).  NaN never culls.
 * cluster_terms: the per-(origin, cluster) values, culled_by: the per-direction test (the chain kernel tabulates
 * the first for a pixel's primary hit point, where every first bounce starts). */
struct ClusterTerms {
    V3 w;
    float w2, A, B; /* T = (A + rho B) * 1.00001 */
};
__device__ __forceinline__ ClusterTerms cluster_terms(V3 pos, const DevCluster &K)
{
    ClusterTerms t;
    t.w = sub(V3{K.cx, K.cy, K.cz}, pos);
    const float S = fabsf(t.w.x) + fabsf(t.w.y) + fabsf(t.w.z) + K.r; /* >= |pos - A| for every vertex A */
    t.w2 = fmaf(t.w.z, t.w.z, fmaf(t.w.y, t.w.y, t.w.x * t.w.x));
    t.A = (K.r + kClusterGamma * S) + K.gammaE;
    t.B = fmaf(K.beta, S, K.alpha);
    return t;
}
__device__ __forceinline__ bool culled_by(const ClusterTerms &t, V3 dir, float rho, float dd)
{
    const float T = fmaf(rho, t.B, t.A) * 1.00001f;
    const float T2 = T * T;
    const float b = fmaf(t.w.z, dir.z, fmaf(t.w.y, dir.y, t.w.x * dir.x));
    const float wd = t.w2 * dd;
    const float x2 = fmaf(-b, b, wd);
    return b > 0.f ? (x2 - 1.5e-6f * wd > T2 * dd) : (t.w2 > T2);
}
__device__ __forceinline__ float dir_dd(V3 dir) { return fmaf(dir.z, dir.z, fmaf(dir.y, dir.y, dir.x * dir.x)); }
__device__ __forceinline__ bool cluster_culled(V3 pos, V3 dir, float rho, float dd, const DevCluster &K)
{
    return culled_by(cluster_terms(pos, K), dir, rho, dd);
}

__host__ __device__ static inline V3 v3(vec3 v) { return V3{v.x, v.y, v.z}; }

/* the tile cull keeps a workgroup's prefilter survivors in LDS (maskWords u64, <= 48 KB: 393,216 triangles); larger
 * scenes render without it, and without the geometry kernel whose occupancy bounce_hit_share chooses */
constexpr int kMaxCullMaskWords = 6144;

/*
 * rtc_probe.hip -- the reference's single functions on the device for known-answer tests (include/rtc.h rtc_probe_*):
 * rayTriangle (raytracing.c:186-214), raySphere (:162-184), getEnvironmentLight (:151-160), the RNG
 * (moremath.c:89-108), and the soundness probe of the bounce-ray cluster culling (rtc_layout.h cluster_culled).
 */
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "rtc_layout.h"
#include "rtc_internal.h"
#include "rtc_hip_util.h"

/* ---- probes: single reference functions on the device, for known-answer tests ---------------------- */
__global__ void probe_tri_kernel(const Ray *rays, const Triangle *tris, size_t n, int *didHit, float *dst)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const Ray R = rays[i];
    const Triangle T = tris[i];
    const V3 A = v3(T.posA);
    float d = 0.f;
    bool h = ray_triangle(v3(R.pos), v3(R.dir), A, sub(v3(T.posB), A), sub(v3(T.posC), A), v3(T.normal), d);
    didHit[i] = h ? 1 : 0;
    dst[i] = h ? d : 0.f;
}

__global__ void probe_sphere_kernel(const Ray *rays, const Sphere *sph, size_t n, int *didHit, float *dst,
                                    vec3 *normal)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const Ray R = rays[i];
    const Sphere S = sph[i];
    float d = 0.f;
    bool h = ray_sphere(v3(R.pos), v3(R.dir), v3(S.pos), S.r, d);
    didHit[i] = h ? 1 : 0;
    dst[i] = h ? d : 0.f;
    V3 nrm{0.f, 0.f, 0.f};
    if (h)
        nrm = normalized(sub(add(v3(R.pos), mul(v3(R.dir), d)), v3(S.pos)));
    normal[i] = vec3{nrm.x, nrm.y, nrm.z};
}

__global__ void probe_env_kernel(const Ray *rays, const Scene *scenes, size_t n, vec3 *out)
{
    __shared__ PowTablesLds sPow; /* the environment reads its powf tables from LDS, as in the render kernels */
    sPow.fill(threadIdx.x);
    __syncthreads();
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    Scene s = scenes[i];
    EnvParams e{};
    sPow.attach(e);
    e.sun = v3(s.normalizedSunDirection);
    e.horizon = v3(s.skyColorHorizon);
    e.zenith = v3(s.skyColorZenith);
    e.ground = v3(s.groundColor);
    e.focus = s.sunFocus;
    e.intensity = s.sunIntensity;
    e.sunSkip = env_sun_skippable(e.focus, e.intensity);
    V3 c = environment(v3(rays[i].dir), e);
    out[i] = vec3{c.x, c.y, c.z};
}

__host__ __device__ static double rtc_env_vanish_limit_of(const Scene &s)
{
    const float col[9] = {s.groundColor.x,     s.groundColor.y,     s.groundColor.z,
                          s.skyColorHorizon.x, s.skyColorHorizon.y, s.skyColorHorizon.z,
                          s.skyColorZenith.x,  s.skyColorZenith.y,  s.skyColorZenith.z};
    return env_vanish_limit(s.sunFocus, s.sunIntensity, col);
}

/* the sky kernel's per-pixel sun skip (rtc_device.h sun_vanishes) and the environment evaluated with it */
__global__ void probe_vanish_kernel(const Ray *rays, const Scene *scenes, size_t n, int *vanish, vec3 *out)
{
    __shared__ PowTablesLds sPow;
    sPow.fill(threadIdx.x);
    __syncthreads();
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const Scene s = scenes[i];
    EnvParams e{};
    sPow.attach(e);
    e.sun = v3(s.normalizedSunDirection);
    e.horizon = v3(s.skyColorHorizon);
    e.zenith = v3(s.skyColorZenith);
    e.ground = v3(s.groundColor);
    e.focus = s.sunFocus;
    e.intensity = s.sunIntensity;
    e.sunSkip = env_sun_skippable(e.focus, e.intensity);
    e.vanishLim = rtc_env_vanish_limit_of(s);
    const V3 d = v3(rays[i].dir);
    const bool v = sun_vanishes(d, e);
    vanish[i] = v ? 1 : 0;
    const V3 c = environment_t<false>(d, e, v);
    out[i] = vec3{c.x, c.y, c.z};
}

__global__ void probe_random_kernel(const unsigned *seeds, size_t n, int draws, float *uni, float *nrm, vec3 *dirs)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    unsigned s = seeds[i];
    for (int k = 0; k < draws; ++k)
        uni[i * draws + k] = random_value(s);
    s = seeds[i];
    for (int k = 0; k < draws; ++k)
        nrm[i * draws + k] = random_normal(s);
    s = seeds[i];
    for (int k = 0; k < draws; ++k) {
        V3 d = random_direction(s);
        dirs[i * draws + k] = vec3{d.x, d.y, d.z};
    }
}

/* Cluster culling soundness (DevCluster): every (ray, cluster) pair is culled or not by cluster_culled, and
 * every triangle of the cluster is tested with the reference's rayTriangle arithmetic.  counts: [0] hits in
 * culled clusters (must stay 0), [1] clusters culled, [2] cluster tests, [3] hits, [4] float bits of the
 * largest (distance from the ball centre to the reported hit point) - r over all hits; with reach, [5] hits on
 * records judged unreachable from the ray's origin (aligned_normal; must stay 0), [6] (ray, record) pairs judged
 * so. */
__global__ void probe_cluster_kernel(const DevTri *clTris, const DevCluster *cl, int clusterCount, int per,
                                     int recCount, bool reach, const Ray *rays, size_t n,
                                     unsigned long long *counts)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const V3 pos = v3(rays[i].pos), dir = v3(rays[i].dir);
    const float rho = fabsf(dir.x) + fabsf(dir.y) + fabsf(dir.z);
    unsigned viol = 0, culled = 0, hits = 0, unreachHits = 0, unreach = 0;
    float excess = 0.f;
    for (int k = 0; k < clusterCount; ++k) {
        const DevCluster K = cl[k];
        const bool cut = rho <= kClusterRhoMax && cluster_culled(pos, dir, rho, dir_dd(dir), K);
        culled += cut;
        for (int j = 0; j < per && k * per + j < recCount; ++j) {
            const DevTri R = clTris[k * per + j];
            if (__float_as_int(R.pad0) < 0)
                continue;
            /* rtc_render_chain's first-bounce reach mask: not hittable from pos in any direction */
            const V3 q = cross(sub(pos, V3{R.ax, R.ay, R.az}), V3{R.abx, R.aby, R.abz});
            const bool cannot = reach && rho <= kClusterRhoMax && __float_as_int(R.pad1) != 0 &&
                                !(dot(V3{R.acx, R.acy, R.acz}, q) > 0.f);
            unreach += cannot;
            float dst;
            if (ray_triangle(pos, dir, V3{R.ax, R.ay, R.az}, V3{R.abx, R.aby, R.abz}, V3{R.acx, R.acy, R.acz},
                             V3{R.nx, R.ny, R.nz}, dst)) {
                hits++;
                viol += cut;
                unreachHits += cannot;
                const V3 h = add(pos, mul(dir, dst));
                const V3 w = sub(h, V3{K.cx, K.cy, K.cz});
                excess = fmaxf(excess, (float)__builtin_sqrt((double)dot(w, w)) - K.r);
            }
        }
    }
    atomicAdd(&counts[0], (unsigned long long)viol);
    atomicAdd(&counts[1], (unsigned long long)culled);
    atomicAdd(&counts[2], (unsigned long long)clusterCount);
    atomicAdd(&counts[3], (unsigned long long)hits);
    atomicMax(&counts[4], (unsigned long long)__float_as_uint(excess));
    if (reach) {
        atomicAdd(&counts[5], (unsigned long long)unreachHits);
        atomicAdd(&counts[6], (unsigned long long)unreach);
    }
}

namespace {
struct Scratch {
    std::vector<void *> ptrs;
    ~Scratch()
    {
        for (void *p : ptrs)
            (void)hipFree(p);
    }
    hipError_t alloc(void **p, size_t bytes)
    {
        hipError_t e = hipMalloc(p, bytes ? bytes : 16);
        if (e == hipSuccess)
            ptrs.push_back(*p);
        return e;
    }
};
int probe_prelude()
{
    int n = 0;
    return rtc_device_count(&n);
}
} // namespace

#define ALLOC_IN(dptr, hptr, bytes)                                                                    \
    HIP_TRY(sc.alloc((void **)&dptr, bytes));                                                          \
    HIP_TRY(hipMemcpy(dptr, hptr, bytes, hipMemcpyHostToDevice))
#define ALLOC_OUT(dptr, bytes) HIP_TRY(sc.alloc((void **)&dptr, bytes))

static unsigned probe_blocks(size_t n) { return (unsigned)((n + 255) / 256 > 0 ? (n + 255) / 256 : 1); }

extern "C" int rtc_probe_ray_triangle(const Ray *rays, const Triangle *tris, size_t n, int *didHit, float *dst)
{
    if (int rc = probe_prelude())
        return rc;
    if (n == 0)
        return 0;
    Scratch sc;
    Ray *dr;
    Triangle *dt;
    int *dh;
    float *dd;
    ALLOC_IN(dr, rays, n * sizeof(Ray));
    ALLOC_IN(dt, tris, n * sizeof(Triangle));
    ALLOC_OUT(dh, n * sizeof(int));
    ALLOC_OUT(dd, n * sizeof(float));
    hipLaunchKernelGGL(probe_tri_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, dr, dt, n, dh, dd);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(didHit, dh, n * sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(dst, dd, n * sizeof(float), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int rtc_probe_ray_sphere(const Ray *rays, const Sphere *spheres, size_t n, int *didHit, float *dst,
                                    vec3 *normal)
{
    if (int rc = probe_prelude())
        return rc;
    if (n == 0)
        return 0;
    Scratch sc;
    Ray *dr;
    Sphere *ds;
    int *dh;
    float *dd;
    vec3 *dn;
    ALLOC_IN(dr, rays, n * sizeof(Ray));
    ALLOC_IN(ds, spheres, n * sizeof(Sphere));
    ALLOC_OUT(dh, n * sizeof(int));
    ALLOC_OUT(dd, n * sizeof(float));
    ALLOC_OUT(dn, n * sizeof(vec3));
    hipLaunchKernelGGL(probe_sphere_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, dr, ds, n, dh, dd, dn);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(didHit, dh, n * sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(dst, dd, n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(normal, dn, n * sizeof(vec3), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int rtc_probe_environment(const Ray *rays, const Scene *scenes, size_t n, vec3 *out)
{
    if (int rc = probe_prelude())
        return rc;
    if (n == 0)
        return 0;
    Scratch sc;
    Ray *dr;
    Scene *ds;
    vec3 *dout;
    ALLOC_IN(dr, rays, n * sizeof(Ray));
    ALLOC_IN(ds, scenes, n * sizeof(Scene));
    ALLOC_OUT(dout, n * sizeof(vec3));
    hipLaunchKernelGGL(probe_env_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, dr, ds, n, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, n * sizeof(vec3), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int rtc_probe_sun_vanish(const Ray *rays, const Scene *scenes, size_t n, int *vanish, vec3 *out)
{
    if (int rc = probe_prelude())
        return rc;
    if (n == 0)
        return 0;
    Scratch sc;
    Ray *dr;
    Scene *ds;
    int *dv;
    vec3 *dout;
    ALLOC_IN(dr, rays, n * sizeof(Ray));
    ALLOC_IN(ds, scenes, n * sizeof(Scene));
    ALLOC_OUT(dv, n * sizeof(int));
    ALLOC_OUT(dout, n * sizeof(vec3));
    hipLaunchKernelGGL(probe_vanish_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, dr, ds, n, dv, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(vanish, dv, n * sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out, dout, n * sizeof(vec3), hipMemcpyDeviceToHost));
    return 0;
}

/* the limit sun_vanishes compares with (host code: no device needed) */
extern "C" int rtc_env_vanish_limit(const Scene *scene, double *limit)
{
    if (!scene || !limit)
        return RTC_EINVAL;
    *limit = rtc_env_vanish_limit_of(*scene);
    return 0;
}

extern "C" int rtc_probe_random(const unsigned int *seeds, size_t n, int draws, float *uniform, float *normal,
                                vec3 *direction)
{
    if (int rc = probe_prelude())
        return rc;
    if (n == 0 || draws <= 0)
        return 0;
    Scratch sc;
    unsigned *dsd;
    float *du, *dn;
    vec3 *dd;
    const size_t m = n * (size_t)draws;
    ALLOC_IN(dsd, seeds, n * sizeof(unsigned));
    ALLOC_OUT(du, m * sizeof(float));
    ALLOC_OUT(dn, m * sizeof(float));
    ALLOC_OUT(dd, m * sizeof(vec3));
    hipLaunchKernelGGL(probe_random_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, dsd, n, draws, du, dn, dd);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(uniform, du, m * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(normal, dn, m * sizeof(float), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(direction, dd, m * sizeof(vec3), hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int rtc_probe_cluster_bound(const Triangle *tris, int triCount, const Ray *rays, size_t n,
                                       unsigned long long counts[7])
{
    if (!counts || triCount < 0 || (triCount > 0 && !tris) || (n > 0 && !rays))
        return rtc_fail(RTC_EINVAL, "rtc_probe_cluster_bound: bad argument");
    memset(counts, 0, 7 * sizeof(unsigned long long));
    if (int rc = probe_prelude())
        return rc;
    if (n == 0 || triCount == 0)
        return 0;
    RtcDeviceScene *s = nullptr;
    if (int rc = rtc_scene_upload(tris, triCount, nullptr, 0, -1, &s))
        return rc;
    Scratch sc;
    Ray *dr = nullptr;
    unsigned long long *dc = nullptr;
    int rc = 0;
    hipError_t e = sc.alloc((void **)&dr, n * sizeof(Ray));
    if (e == hipSuccess)
        e = hipMemcpy(dr, rays, n * sizeof(Ray), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = sc.alloc((void **)&dc, 7 * sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMemset(dc, 0, 7 * sizeof(unsigned long long));
    if (e == hipSuccess) {
        /* the clusters, then the chunks (balls over kChunkClusters clusters, rtc_render_chain's first level) */
        hipLaunchKernelGGL(probe_cluster_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, s->clTris, s->clusters,
                           s->clusterCount, kClusterSize, s->clusterCount * kClusterSize, true, dr, n, dc);
        e = hipGetLastError();
        if (e == hipSuccess && s->chunkCount > 1) {
            hipLaunchKernelGGL(probe_cluster_kernel, dim3(probe_blocks(n)), dim3(256), 0, nullptr, s->clTris, s->chunks,
                               s->chunkCount, kClusterSize * kChunkClusters, s->clusterCount * kClusterSize, false, dr, n,
                               dc);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess)
        e = hipMemcpy(counts, dc, 7 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    if (e != hipSuccess)
        rc = rtc_fail(-(int)e, "rtc_probe_cluster_bound: %s", hipGetErrorString(e));
    rtc_scene_release(s);
    return rc;
}

/*
 * rtc_scene.hip -- the scene on the device (rtc_scene_upload / rtc_scene_release, include/rtc.h): the reference's
 * Triangle[] (objloader.c / main.c:229-243) packed into the HBM records of rtc_layout.h, grouped into clusters and chunks
 * for the bounce rays' culling, the scheduling hint bounce_hit_share, the scene's streams and ordering events, and the
 * per-scene hooks (frame / geometry events, kernel timing).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "rtc_layout.h"
#include "rtc_internal.h"
#include "rtc_hip_util.h"

/* The share of diffuse bounce rays that hit the scene again, estimated at upload (host, a fixed-seed probe): rays from
 * area-weighted random points of the triangles, in directions normal + a random unit vector (the reference's diffuse
 * lobe, raytracing.c:276-279, without the specular part), tested against every triangle in double precision with the
 * reference's backface rule.  Only a scheduling hint (rtc_render_chain's workgroups per CU): it never changes a
 * frame.  Measured shares: fsuzane 0.21, rsuzanne 0.11, ultracomplex 0.019, complex 0.016, cube 0. */
static double bounce_hit_share(const Triangle *t, int n)
{
    if (n <= 0)
        return 0.0;
    struct D3 { double x, y, z; };
    const auto sub3 = [](D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; };
    const auto dot3 = [](D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
    const auto cross3 = [](D3 a, D3 b) { return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; };
    const auto d3 = [](vec3 v) { return D3{v.x, v.y, v.z}; };
    std::vector<double> cdf((size_t)n);
    double total = 0.0;
    for (int i = 0; i < n; ++i) {
        const D3 c = cross3(sub3(d3(t[i].posB), d3(t[i].posA)), sub3(d3(t[i].posC), d3(t[i].posA)));
        total += 0.5 * std::sqrt(dot3(c, c));
        cdf[(size_t)i] = total;
    }
    if (!(total > 0.0))
        return 0.0;
    unsigned long long st = 0x9E3779B97F4A7C15ull;
    const auto uni = [&]() { /* xorshift64*, [0, 1) */
        st ^= st >> 12;
        st ^= st << 25;
        st ^= st >> 27;
        return (double)((st * 0x2545F4914F6CDD1Dull) >> 11) * (1.0 / 9007199254740992.0);
    };
    /* rays x n ray-triangle tests: ~4 M up to 62.5 k triangles, 64 n beyond (a 1 M-triangle scene: 64 M tests, a few
     * tenths of a second of upload; scenes past the tile cull's limit skip the probe, rtc_scene_upload) */
    const int rays = (int)std::min<long long>(2048, std::max<long long>(64, 4000000LL / n));
    int hits = 0;
    for (int r = 0; r < rays; ++r) {
        const int i = (int)(std::lower_bound(cdf.begin(), cdf.end(), uni() * total) - cdf.begin());
        const Triangle &T = t[std::min(i, n - 1)];
        double u = uni(), w = uni();
        if (u + w > 1.0) {
            u = 1.0 - u;
            w = 1.0 - w;
        }
        const D3 A = d3(T.posA), AB = sub3(d3(T.posB), A), AC = sub3(d3(T.posC), A);
        D3 nn = d3(T.normal);
        const double nl = std::sqrt(dot3(nn, nn));
        if (!(nl > 0.0))
            continue;
        nn = D3{nn.x / nl, nn.y / nl, nn.z / nl};
        D3 q{0, 0, 0};
        double ql = 0.0;
        do { /* a uniform random unit vector (rejection from the cube) */
            q = D3{2 * uni() - 1, 2 * uni() - 1, 2 * uni() - 1};
            ql = dot3(q, q);
        } while (ql > 1.0 || ql < 1e-12);
        ql = std::sqrt(ql);
        D3 dir{nn.x + q.x / ql, nn.y + q.y / ql, nn.z + q.z / ql};
        const double dl = std::sqrt(dot3(dir, dir));
        if (!(dl > 1e-9))
            continue;
        dir = D3{dir.x / dl, dir.y / dl, dir.z / dl};
        const D3 P{A.x + u * AB.x + w * AC.x + 1e-4 * nn.x, A.y + u * AB.y + w * AC.y + 1e-4 * nn.y,
                   A.z + u * AB.z + w * AC.z + 1e-4 * nn.z};
        for (int j = 0; j < n; ++j) { /* rayTriangle's tests (raytracing.c:186-214), in double */
            if (dot3(dir, d3(t[j].normal)) >= 0.0)
                continue;
            const D3 a = d3(t[j].posA), ab = sub3(d3(t[j].posB), a), ac = sub3(d3(t[j].posC), a);
            const D3 h = cross3(dir, ac);
            const double det = dot3(ab, h);
            if (std::fabs(det) < 1e-12)
                continue;
            const D3 sv = sub3(P, a);
            const double uu = dot3(sv, h) / det;
            if (uu < 0.0 || uu > 1.0)
                continue;
            const D3 qv = cross3(sv, ab);
            const double vv = dot3(dir, qv) / det;
            if (vv < 0.0 || uu + vv > 1.0 || dot3(ac, qv) / det < 1e-3)
                continue;
            ++hits;
            break;
        }
    }
    return (double)hits / (double)rays;
}

static void pack_scene(const Triangle *tris, int triCount, const Sphere *sph, int sphCount, std::vector<DevTri> &dt,
                       std::vector<DevMat> &dm, std::vector<DevSphere> &ds)
{
    const size_t padded = ((size_t)(triCount > 0 ? triCount : 0) + 7) / 8 * 8 + 8;
    /* zero records are never hit: N = 0 makes dot(dir, N) >= 0 (or NaN, and then det is NaN too) */
    dt.assign(padded, DevTri{});
    dm.assign(padded, DevMat{});
    for (int i = 0; i < triCount; ++i) {
        const Triangle &t = tris[i];
        DevTri &d = dt[i];
        memset(&d, 0, sizeof d);
        d.ax = t.posA.x;
        d.ay = t.posA.y;
        d.az = t.posA.z;
        /* raytracing.c:191-192 minus(posB, posA), minus(posC, posA): same f32 ops */
        d.abx = t.posB.x - t.posA.x;
        d.aby = t.posB.y - t.posA.y;
        d.abz = t.posB.z - t.posA.z;
        d.acx = t.posC.x - t.posA.x;
        d.acy = t.posC.y - t.posA.y;
        d.acz = t.posC.z - t.posA.z;
        d.nx = t.normal.x;
        d.ny = t.normal.y;
        d.nz = t.normal.z;
        DevMat &m = dm[i];
        memset(&m, 0, sizeof m);
        m.r = t.mat.color.x;
        m.g = t.mat.color.y;
        m.b = t.mat.color.z;
        m.emission = t.mat.emissionStrength;
        m.smoothness = t.mat.smoothness;
    }
    ds.resize(sphCount > 0 ? sphCount : 1);
    for (int i = 0; i < sphCount; ++i) {
        DevSphere &d = ds[i];
        memset(&d, 0, sizeof d);
        d.cx = sph[i].pos.x;
        d.cy = sph[i].pos.y;
        d.cz = sph[i].pos.z;
        d.radius = sph[i].r;
        d.r = sph[i].mat.color.x;
        d.g = sph[i].mat.color.y;
        d.b = sph[i].mat.color.z;
        d.emission = sph[i].mat.emissionStrength;
        d.smoothness = sph[i].mat.smoothness;
    }
}

/* Clusters of kClusterSize triangles: recursive splits of the centroids along their longest extent, each
 * split at a multiple of kClusterSize so that every leaf but the last is full (ceil(n / 8) clusters). */
static void split_clusters(const std::vector<DevTri> &dt, std::vector<int> &idx, size_t lo, size_t hi)
{
    const size_t n = hi - lo;
    if (n <= (size_t)kClusterSize)
        return;
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    auto centroid = [&](int i, int a) {
        const DevTri &t = dt[i];
        const double A[3] = {t.ax, t.ay, t.az}, B[3] = {t.abx, t.aby, t.abz}, C[3] = {t.acx, t.acy, t.acz};
        return A[a] + (B[a] + C[a]) / 3.0;
    };
    for (size_t k = lo; k < hi; ++k)
        for (int a = 0; a < 3; ++a) {
            const double c = centroid(idx[k], a);
            if (c == c) {
                mn[a] = std::min(mn[a], c);
                mx[a] = std::max(mx[a], c);
            }
        }
    int axis = 0;
    for (int a = 1; a < 3; ++a)
        if (mx[a] - mn[a] > mx[axis] - mn[axis])
            axis = a;
    std::stable_sort(idx.begin() + lo, idx.begin() + hi, [&](int p, int q) {
        const double cp = centroid(p, axis), cq = centroid(q, axis);
        return (cp == cp ? cp : 1e300) < (cq == cq ? cq : 1e300);
    });
    const size_t leaves = (n + kClusterSize - 1) / kClusterSize;
    const size_t mid = lo + (leaves + 1) / 2 * kClusterSize;
    split_clusters(dt, idx, lo, mid);
    split_clusters(dt, idx, mid, hi);
}

/* Bounding ball and cull margins (DevCluster) of the records ct[first, first + count) whose index (pad0) is
 * >= 0: the ball holds every vertex A, A + AB, A + AC; E is the longest AB / AC edge. */
static DevCluster ball_of(const std::vector<DevTri> &ct, size_t first, size_t count)
{
    const double u = 0x1p-24, eps = 0.001; /* |det| >= 0.001f > 0.001 for every reported hit */
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, E = 0.0;
    bool finite = true;
    int n = 0;
    auto real = [&](const DevTri &r) {
        int i;
        memcpy(&i, &r.pad0, sizeof i);
        return i >= 0;
    };
    for (size_t j = first; j < first + count; ++j) {
        const DevTri &r = ct[j];
        if (!real(r))
            continue;
        ++n;
        const double A[3] = {r.ax, r.ay, r.az}, B[3] = {r.abx, r.aby, r.abz}, C[3] = {r.acx, r.acy, r.acz};
        for (int a = 0; a < 3; ++a) {
            const double v[3] = {A[a], A[a] + B[a], A[a] + C[a]};
            for (double x : v) {
                finite = finite && std::isfinite(x);
                lo[a] = std::min(lo[a], x);
                hi[a] = std::max(hi[a], x);
            }
        }
        E = std::max(E, std::max(std::sqrt(B[0] * B[0] + B[1] * B[1] + B[2] * B[2]),
                                 std::sqrt(C[0] * C[0] + C[1] * C[1] + C[2] * C[2])));
    }
    DevCluster k{};
    const double ctr[3] = {(lo[0] + hi[0]) / 2, (lo[1] + hi[1]) / 2, (lo[2] + hi[2]) / 2};
    k.cx = n ? (float)ctr[0] : 0.f;
    k.cy = n ? (float)ctr[1] : 0.f;
    k.cz = n ? (float)ctr[2] : 0.f;
    double R = 0.0;
    for (size_t j = first; j < first + count; ++j) { /* radius about the rounded (float) centre */
        const DevTri &r = ct[j];
        if (!real(r))
            continue;
        const double A[3] = {r.ax, r.ay, r.az}, B[3] = {r.abx, r.aby, r.abz}, C[3] = {r.acx, r.acy, r.acz};
        const double K[3] = {k.cx, k.cy, k.cz};
        for (int w = 0; w < 3; ++w) {
            double d2 = 0.0;
            for (int a = 0; a < 3; ++a) {
                const double x = A[a] + (w == 1 ? B[a] : w == 2 ? C[a] : 0.0) - K[a];
                d2 += x * x;
            }
            R = std::max(R, std::sqrt(d2));
        }
    }
    const double F = 4.0, edRatio = 8.0 * u * E * E * kClusterRhoMax / eps;
    k.r = std::nextafter((float)(R * (1.0 + 1e-9)), INFINITY);
    k.e = (float)E;
    if (!finite || n == 0 || !(edRatio < 0.5) || !(k.r < 1e18f)) {
        k.alpha = INFINITY; /* never culled */
        k.beta = k.gammaE = 0.f;
        return k;
    }
    const double kk = 1.0 / (1.0 - edRatio);
    k.alpha = std::nextafter((float)(F * kk * 32.0 * u * E * E * E / eps), INFINITY);
    k.beta = std::nextafter((float)(F * kk * 45.0 * u * E * E / eps), INFINITY);
    k.gammaE = std::nextafter((float)(kClusterGamma * E), INFINITY);
    return k;
}

/* A triangle whose stored normal N points along its geometric normal G' = AB x AC closely enough that, for every
 * ray of |dir|_1 <= kClusterRhoMax, rayTriangle's backface test (dot(dir, N) < 0, raytracing.c:189) forces
 * det = dot(AB, dir x AC) > -EPSILON (raytracing.c:195): then a hit needs det >= EPSILON, and since
 * dst = dot(AC, q) / det (q = (pos - A) x AB, raytracing.c:202-206) must be >= EPSILON, dot(AC, q) > 0.  For a
 * ray origin where the reference's own f32 dot(AC, q) is <= 0 (pos on or behind the plane), the triangle cannot
 * be hit from there in any direction (rtc_render_chain's first bounces).  Bound: with N = a G'/|G'| + e (e
 * orthogonal), fl(dot(dir, N)) < 0 gives dir.G'/|G'| < rho (3.01u |N|_inf + |e|) / a, and |det + dir.G'| <=
 * 5.1u |AB|_1 |AC|_1 rho; aligned when rho times their sum, with a factor 2, stays below EPSILON. */
static bool aligned_normal(const DevTri &r)
{
    const double u = 0x1p-24;
    const double AB[3] = {r.abx, r.aby, r.abz}, AC[3] = {r.acx, r.acy, r.acz}, N[3] = {r.nx, r.ny, r.nz};
    const double G[3] = {AB[1] * AC[2] - AB[2] * AC[1], AB[2] * AC[0] - AB[0] * AC[2], AB[0] * AC[1] - AB[1] * AC[0]};
    const double g = std::sqrt(G[0] * G[0] + G[1] * G[1] + G[2] * G[2]);
    if (!(g > 0.0) || !std::isfinite(g))
        return false;
    const double a = (N[0] * G[0] + N[1] * G[1] + N[2] * G[2]) / g;
    if (!(a > 0.0))
        return false;
    const double e[3] = {N[0] - a * G[0] / g, N[1] - a * G[1] / g, N[2] - a * G[2] / g};
    const double en = std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]) + 1e-12 * (std::fabs(N[0]) + std::fabs(N[1]) + std::fabs(N[2]));
    const double ninf = std::max(std::fabs(N[0]), std::max(std::fabs(N[1]), std::fabs(N[2])));
    const double n1 = std::fabs(AB[0]) + std::fabs(AB[1]) + std::fabs(AB[2]), c1 = std::fabs(AC[0]) + std::fabs(AC[1]) + std::fabs(AC[2]);
    const double K = g * (3.01 * u * ninf + en) / a + 5.1 * u * n1 * c1;
    return std::isfinite(K) && 2.0 * kClusterRhoMax * K < 0.001;
}

/* ct: the records in cluster order (pad0 = reference index, -1 for padding), cl: one ball per cluster of
 * kClusterSize, ch: one ball per chunk of kChunkClusters consecutive clusters (a subtree of the median split:
 * the chain kernel's first culling level for scenes of more than one chunk) */
static void rtc_build_clusters(const std::vector<DevTri> &dt, int triCount, std::vector<DevTri> &ct,
                               std::vector<DevCluster> &cl, std::vector<DevCluster> &ch)
{
    const int nc = (triCount + kClusterSize - 1) / kClusterSize;
    std::vector<int> idx(triCount);
    for (int i = 0; i < triCount; ++i)
        idx[i] = i;
    split_clusters(dt, idx, 0, (size_t)triCount);
    ct.assign((size_t)nc * kClusterSize, DevTri{});
    cl.assign((size_t)(nc > 0 ? nc : 1), DevCluster{});
    for (int c = 0; c < nc; ++c) {
        const int n = std::min(kClusterSize, triCount - c * kClusterSize);
        for (int j = 0; j < kClusterSize; ++j) {
            DevTri &r = ct[(size_t)c * kClusterSize + j];
            if (j >= n) { /* zero record: never hit; index -1 */
                const int none = -1;
                memcpy(&r.pad0, &none, sizeof none);
                continue;
            }
            const int i = idx[(size_t)c * kClusterSize + j];
            r = dt[i];
            memcpy(&r.pad0, &i, sizeof i);
            const int al = aligned_normal(r) ? 1 : 0;
            memcpy(&r.pad1, &al, sizeof al);
        }
        cl[c] = ball_of(ct, (size_t)c * kClusterSize, kClusterSize);
    }
    const int nch = (nc + kChunkClusters - 1) / kChunkClusters;
    ch.assign((size_t)(nch > 0 ? nch : 1), DevCluster{});
    for (int h = 0; h < nch; ++h) {
        const size_t c0 = (size_t)h * kChunkClusters, c1 = std::min<size_t>((size_t)nc, c0 + kChunkClusters);
        ch[h] = ball_of(ct, c0 * kClusterSize, (c1 - c0) * kClusterSize);
    }
}

extern "C" int rtc_bounce_hit_share(const Triangle *tris, int triCount, float *share)
{
    if (!share || triCount < 0 || (triCount > 0 && !tris))
        return rtc_fail(RTC_EINVAL, "rtc_bounce_hit_share: bad argument");
    *share = (float)bounce_hit_share(tris, triCount);
    return 0;
}

extern "C" int rtc_scene_chain_wgs(const RtcDeviceScene *s)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "rtc_scene_chain_wgs: null scene");
    return s->chainWgsFull;
}

extern "C" int rtc_scene_upload(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount, int device,
                                RtcDeviceScene **out)
{
    return rtc_scene_upload_with_share(tris, triCount, spheres, sphereCount, device, -1.f, out);
}


extern "C" float rtc_upload_hit_share(const Triangle *tris, int triCount)
{
    const int maskWords = ((triCount + 7) / 8 * 8 + 63) / 64;
    return triCount > 0 && tris && maskWords <= kMaxCullMaskWords ? (float)bounce_hit_share(tris, triCount) : 0.f;
}

extern "C" int rtc_scene_upload_with_share(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                                           int device, float hitShare, RtcDeviceScene **out)
{
    if (!out || triCount < 0 || sphereCount < 0 || (triCount > 0 && !tris) || (sphereCount > 0 && !spheres))
        return rtc_fail(RTC_EINVAL, "rtc_scene_upload: bad argument");
    *out = nullptr;
    int n = 0;
    int rc = rtc_device_count(&n);
    if (rc)
        return rc;
    if (device < 0)
        HIP_TRY(hipGetDevice(&device));
    if (device >= n)
        return rtc_fail(RTC_EINVAL, "device %d out of range (%d devices)", device, n);
    RtcDeviceGuard guard(device);
    if (!guard.ok())
        return rtc_fail(RTC_ENODEV, "rtc_scene_upload: cannot select device %d", device);
    std::vector<DevTri> dt;
    std::vector<DevMat> dm;
    std::vector<DevSphere> ds;
    pack_scene(tris, triCount, spheres, sphereCount, dt, dm, ds);
    std::vector<DevTri> ct;
    std::vector<DevCluster> cl, ch;
    rtc_build_clusters(dt, triCount, ct, cl, ch);
    if (ct.empty())
        ct.assign(1, DevTri{});
    RtcDeviceScene *s = new RtcDeviceScene();
    s->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256; /* MI355X */
    s->cuCount = cus;
    s->triCount = triCount;
    s->triPadded = (triCount + 7) / 8 * 8; /* whole pairs of batches; arrays hold 8 more records for prefetch */
    s->sphereCount = sphereCount;
    s->maskWords = (s->triPadded + 63) / 64;
    s->clusterCount = (triCount + kClusterSize - 1) / kClusterSize;
    s->chunkCount = (s->clusterCount + kChunkClusters - 1) / kChunkClusters;
    /* whole frames of scenes whose bounce rays often hit again (fsuzane) run 4 chain workgroups per CU: their frame is
     * nearly all geometry kernel, which then has the registers the co-resident sky waves would use (round 5, 1080p x64:
     * fsuzane 1.25 -> 1.16 ms per frame; ultracomplex 0.348 -> 0.379, complex 4K 1.22 -> 1.34, so 3 stays the default,
     * profiles/r05_w4_ab_chain_wgs.log) */
    s->hitShare = hitShare >= 0.f ? (double)hitShare : (double)rtc_upload_hit_share(tris, triCount);
    s->chainWgsFull = s->hitShare > kWgsHitShare ? RTC_CHAIN_WGS_HIT : RTC_CHAIN_WGS_FULL;
    hipError_t e = hipMalloc(&s->tris, dt.size() * sizeof(DevTri));
    if (e == hipSuccess)
        e = hipMalloc(&s->clTris, ct.size() * sizeof(DevTri));
    if (e == hipSuccess)
        e = hipMalloc(&s->clusters, cl.size() * sizeof(DevCluster));
    if (e == hipSuccess)
        e = hipMemcpy(s->clTris, ct.data(), ct.size() * sizeof(DevTri), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(s->clusters, cl.data(), cl.size() * sizeof(DevCluster), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMalloc(&s->chunks, ch.size() * sizeof(DevCluster));
    if (e == hipSuccess)
        e = hipMemcpy(s->chunks, ch.data(), ch.size() * sizeof(DevCluster), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMalloc(&s->mats, dm.size() * sizeof(DevMat));
    if (e == hipSuccess)
        e = hipMalloc(&s->spheres, ds.size() * sizeof(DevSphere));
    s->primStride = dt.size();
    if (e == hipSuccess)
        e = hipMalloc(&s->primF, kSkySlots * dt.size() * sizeof(DevPrimF));
    if (e == hipSuccess)
        e = hipMalloc(&s->primX, kSkySlots * dt.size() * sizeof(DevPrimX));
    if (e == hipSuccess)
        e = hipMalloc(&s->segSlots, 256 * 16 * sizeof(unsigned long long));
    if (e == hipSuccess) /* kept zero between launches by rtc_reduce_segments */
        e = hipMemset(s->segSlots, 0, 256 * 16 * sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMalloc(&s->geoCounts, kGeoRing * kGeoSetInts * sizeof(int));
    if (e == hipSuccess)
        e = hipMemset(s->geoCounts, 0, kGeoRing * kGeoSetInts * sizeof(int));
    if (e == hipSuccess)
        e = hipMemcpy(s->tris, dt.data(), dt.size() * sizeof(DevTri), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(s->mats, dm.data(), dm.size() * sizeof(DevMat), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(s->spheres, ds.data(), ds.size() * sizeof(DevSphere), hipMemcpyHostToDevice);
    int leastPrio = 0, greatestPrio = 0;
    if (e == hipSuccess)
        e = hipDeviceGetStreamPriorityRange(&leastPrio, &greatestPrio);
    if (e == hipSuccess) /* the sky tiles yield to the heavy tiles */
        e = hipStreamCreateWithPriority(&s->side, hipStreamNonBlocking, leastPrio);
    if (e == hipSuccess) /* the next frame's cull goes first wherever a CU frees up */
        e = hipStreamCreateWithPriority(&s->cst, hipStreamNonBlocking, greatestPrio);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&s->evCullSync, kOrderEventFlags);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&s->evFork, kOrderEventFlags);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&s->evJoin, kOrderEventFlags);
    for (int h = 0; h < kSkySlots; ++h)
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&s->evSkyDone[h], kOrderEventFlags);
    for (int h = 0; h < kSkySlots; ++h)
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&s->evGeoDone[h], kOrderEventFlags);
    for (hipEvent_t *ev : {&s->evHeavy0, &s->evHeavy1, &s->evSky0, &s->evSky1})
        if (e == hipSuccess)
            e = hipEventCreate(ev);
    if (e != hipSuccess) {
        rtc_scene_release(s);
        return rtc_fail(-(int)e, "scene upload failed: %s", hipGetErrorString(e));
    }
    *out = s;
    return 0;
}

extern "C" int rtc_scene_release(RtcDeviceScene *s)
{
    if (!s)
        return 0;
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(s->device);
    if (s->side) /* an unjoined sky pass (RTC_F_OVERLAP) may still read the scratch */
        (void)hipStreamSynchronize(s->side);
    if (s->cst)
        (void)hipStreamSynchronize(s->cst);
    if (s->cst2)
        (void)hipStreamSynchronize(s->cst2);
    if (s->tris)
        (void)hipFree(s->tris);
    if (s->clTris)
        (void)hipFree(s->clTris);
    if (s->clusters)
        (void)hipFree(s->clusters);
    if (s->chunks)
        (void)hipFree(s->chunks);
    if (s->mats)
        (void)hipFree(s->mats);
    if (s->spheres)
        (void)hipFree(s->spheres);
    if (s->primF)
        (void)hipFree(s->primF);
    if (s->primX)
        (void)hipFree(s->primX);
    if (s->scratch)
        (void)hipFree(s->scratch);
    if (s->samples)
        (void)hipFree(s->samples);
    if (s->segSlots)
        (void)hipFree(s->segSlots);
    if (s->geoCounts)
        (void)hipFree(s->geoCounts);
    if (s->evFork)
        (void)hipEventDestroy(s->evFork);
    if (s->evJoin)
        (void)hipEventDestroy(s->evJoin);
    for (hipEvent_t ev : {s->evHeavy0, s->evHeavy1, s->evSky0, s->evSky1, s->evCullSync})
        if (ev)
            (void)hipEventDestroy(ev);
    for (hipEvent_t ev : s->evSkyDone)
        if (ev)
            (void)hipEventDestroy(ev);
    for (hipEvent_t ev : s->evGeoDone)
        if (ev)
            (void)hipEventDestroy(ev);
    if (s->side)
        (void)hipStreamDestroy(s->side);
    if (s->cst)
        (void)hipStreamDestroy(s->cst);
    if (s->cst2)
        (void)hipStreamDestroy(s->cst2);
    if (cur >= 0)
        (void)hipSetDevice(cur);
    delete s;
    return 0;
}

extern "C" int rtc_rows_selected(const RtcRenderDesc *d)
{
    if (!d || d->rowStride <= 0 || d->rowStart < 0 || d->rowStart >= d->height || d->height <= 0 || d->rowBand < 0)
        return 0;
    /* bands of B rows (rowBand, rtc.h): the full bands' rows, plus the last band's rows inside the frame */
    const long long B = d->rowBand > 1 ? d->rowBand : 1, step = (long long)d->rowStride * B;
    const long long nb = (d->height - d->rowStart + step - 1) / step, last = d->rowStart + (nb - 1) * step;
    return (int)((nb - 1) * B + std::min<long long>(B, d->height - last));
}

extern "C" int rtc_scene_set_geometry_event(RtcDeviceScene *s, void *event)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "rtc_scene_set_geometry_event: null scene");
    s->geoEvent = (hipEvent_t)event;
    return 0;
}

extern "C" int rtc_scene_set_frame_event(RtcDeviceScene *s, void *event)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "rtc_scene_set_frame_event: null scene");
    s->frameEvent = (hipEvent_t)event;
    return 0;
}

extern "C" int rtc_scene_set_timing(RtcDeviceScene *s, int enable)
{
    if (!s)
        return rtc_fail(RTC_EINVAL, "rtc_scene_set_timing: null scene");
    s->timing = enable != 0;
    return 0;
}

extern "C" int rtc_scene_kernel_times(const RtcDeviceScene *s, float out[2])
{
    if (!s || !out)
        return rtc_fail(RTC_EINVAL, "rtc_scene_kernel_times: null argument");
    out[0] = out[1] = -1.f;
    if (!s->timed)
        return 0;
    RtcDeviceGuard guard(s->device);
    HIP_TRY(hipEventSynchronize(s->evHeavy1));
    HIP_TRY(hipEventSynchronize(s->evSky1));
    HIP_TRY(hipEventElapsedTime(&out[0], s->evHeavy0, s->evHeavy1));
    HIP_TRY(hipEventElapsedTime(&out[1], s->evSky0, s->evSky1));
    return 0;
}

/*
 * rtc_frame.hip -- host-buffer renders: the reference's render seam main.c:246-304 as one call.
 *
 *   rtc_render        one device: scene upload, the render launch, and the frame's arrival in host memory
 *   rtc_render_multi  devices 0..G-1 of this process: rows y = g + k*G on device g (the reference's row
 *                     interleave main.c:84 lifted to GPUs), an RCCL gather of the compact parts to device 0
 *                     over xGMI (ncclCommInitAll + ncclGather), the re-interleave on device 0, one D2H
 *
 * Both time the frame as SURVEY.md §8(d) defines it: from the first kernel launch after the scene upload
 * until Color[W*H] is in (pinned) host memory -- the buffer main.c:305 hands to stbi_write_bmp.
 * RtcStats.frameMs is that time; renderMs is the render launch alone (device events).
 *
 * RCCL is opened at run time (dlopen of librccl.so.1: the copy PyTorch-ROCm already holds when torch is
 * loaded, else /opt/rocm's), so single-device users of librtc.so do not pay for loading it.  RCCL errors
 * are returned as positive ncclResult_t codes (SURVEY.md §8 b).
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtc.h"
#include "rtc_hip_util.h"
#include "rtc_internal.h"

namespace {

constexpr size_t kSegBytes = RTC_SEGMENT_COUNTERS * sizeof(unsigned long long);

template <typename T> struct DevBuf {
    T *p = nullptr;
    int device = -1;
    ~DevBuf()
    {
        if (p) {
            RtcDeviceGuard g(device);
            (void)hipFree(p);
        }
    }
    hipError_t alloc(size_t bytes, int dev)
    {
        device = dev;
        return hipMalloc(&p, bytes ? bytes : 16);
    }
};

struct PinnedBuf {
    void *p = nullptr;
    ~PinnedBuf()
    {
        if (p)
            (void)hipHostFree(p);
    }
    hipError_t alloc(size_t bytes) { return hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault); }
};

struct Events {
    std::vector<hipEvent_t> ev;
    ~Events()
    {
        for (hipEvent_t e : ev)
            if (e)
                (void)hipEventDestroy(e);
    }
    hipError_t make(hipEvent_t *out)
    {
        hipError_t e = hipEventCreate(out);
        if (e == hipSuccess)
            ev.push_back(*out);
        return e;
    }
};

double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

/* ---- RCCL, opened at run time -------------------------------------------------------------------- */
struct Rccl {
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    decltype(&ncclCommCount) commCount = nullptr; /* (optional: what each communicator reports, rtc_last_multi_info) */
    bool ok = false;
};

/* What the last rtc_render_multi call of this thread ran on (rtc_last_multi_info): the path, and per
 * communicator the rank count RCCL itself reports (ncclCommCount), so a caller can show that RCCL saw every device */
struct MultiInfo {
    int path = 0; /* 0: no call yet, 1: RCCL gather, 2: host rows (RTC_F_HOST_ROWS, no communicator) */
    int devices = 0;
    std::vector<int> commRanks;
};
thread_local MultiInfo g_multiInfo;

const Rccl &rccl()
{
    static Rccl r = [] {
        Rccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            return x;
        x.commInitAll = (decltype(x.commInitAll))dlsym(h, "ncclCommInitAll");
        x.commDestroy = (decltype(x.commDestroy))dlsym(h, "ncclCommDestroy");
        x.gather = (decltype(x.gather))dlsym(h, "ncclGather");
        x.groupStart = (decltype(x.groupStart))dlsym(h, "ncclGroupStart");
        x.groupEnd = (decltype(x.groupEnd))dlsym(h, "ncclGroupEnd");
        x.errorString = (decltype(x.errorString))dlsym(h, "ncclGetErrorString");
        x.commCount = (decltype(x.commCount))dlsym(h, "ncclCommCount");
        x.ok = x.commInitAll && x.commDestroy && x.gather && x.groupStart && x.groupEnd && x.errorString;
        return x;
    }();
    return r;
}

#define NCCL_TRY(expr)                                                                                 \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess)                                                                         \
            return rtc_fail((int)r_, "%s failed: %s", #expr, rccl().errorString(r_));                  \
    } while (0)

void fill_stats(RtcStats *stats, double renderMs, double frameMs, const unsigned long long *seg, const RtcRenderDesc *d,
                size_t pixels, std::chrono::steady_clock::time_point t0)
{
    if (!stats)
        return;
    stats->renderMs = renderMs;
    stats->frameMs = frameMs;
    stats->segments = seg[0];
    stats->samples = (unsigned long long)pixels * (unsigned long long)(d->spp > 0 ? d->spp : 0);
    stats->triTests = seg[2];
    stats->clusterTests = seg[3];
    stats->discardedTests = seg[4];
    stats->totalMs = ms_since(t0);
}

} // namespace

extern "C" int rtc_render(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                          const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int device,
                          Color *outImage, float *outAccum, RtcStats *stats)
{
    const auto t0 = std::chrono::steady_clock::now();
    if (!scene || !cam || !d || !outImage)
        return rtc_fail(RTC_EINVAL, "rtc_render: null argument");
    int n = 0;
    if (int rc = rtc_device_count(&n))
        return rc;
    if (device < 0)
        HIP_TRY(hipGetDevice(&device));
    if (device >= n)
        return rtc_fail(RTC_EINVAL, "rtc_render: device %d out of range (%d devices)", device, n);
    RtcDeviceGuard guard(device);
    RtcDeviceScene *s = nullptr;
    if (int rc = rtc_scene_upload(tris, triCount, spheres, sphereCount, device, &s))
        return rc;
    struct SceneGuard {
        RtcDeviceScene *s;
        ~SceneGuard() { rtc_scene_release(s); }
    } sceneGuard{s};
    const int rows = rtc_rows_selected(d);
    const size_t px = (size_t)rows * (size_t)(d->width > 0 ? d->width : 0);
    DevBuf<unsigned char> dColors;
    DevBuf<float> dAccum;
    DevBuf<unsigned long long> dSeg;
    PinnedBuf hColors;
    HIP_TRY(dColors.alloc(px * 3 + 16, device));
    if (outAccum)
        HIP_TRY(dAccum.alloc(px * 3 * sizeof(float) + 16, device));
    HIP_TRY(dSeg.alloc(kSegBytes, device));
    HIP_TRY(hipMemset(dSeg.p, 0, kSegBytes));
    HIP_TRY(hColors.alloc(px * 3));
    hipStream_t st = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t st;
        ~StreamGuard() { (void)hipStreamDestroy(st); }
    } streamGuard{st};
    Events evs;
    hipEvent_t e0, e1, e2;
    HIP_TRY(evs.make(&e0));
    HIP_TRY(evs.make(&e1));
    HIP_TRY(evs.make(&e2));
    HIP_TRY(hipEventRecord(e0, st));
    if (int rc = rtc_render_rows_async(s, scene, cam, d, dColors.p, dAccum.p, dSeg.p, st))
        return rc;
    HIP_TRY(hipEventRecord(e1, st));
    /* the frame is done when Color[] is in host memory (main.c:305 consumes it there) */
    HIP_TRY(hipMemcpyAsync(hColors.p, dColors.p, px * 3, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(e2, st));
    HIP_TRY(hipEventSynchronize(e2));
    float renderMs = 0.f, frameMs = 0.f;
    HIP_TRY(hipEventElapsedTime(&renderMs, e0, e1));
    HIP_TRY(hipEventElapsedTime(&frameMs, e0, e2));
    memcpy(outImage, hColors.p, px * 3);
    if (outAccum)
        HIP_TRY(hipMemcpy(outAccum, dAccum.p, px * 3 * sizeof(float), hipMemcpyDeviceToHost));
    unsigned long long seg[RTC_SEGMENT_COUNTERS] = {0};
    HIP_TRY(hipMemcpy(seg, dSeg.p, kSegBytes, hipMemcpyDeviceToHost));
    fill_stats(stats, renderMs, frameMs, seg, d, px, t0);
    return 0;
}

int rtc_render_multi_host_rows(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                               const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int G,
                               Color *outImage, float *outAccum, RtcStats *stats, std::chrono::steady_clock::time_point t0);

/* Part g of G of a full frame d: rows y = g + k*G, or the bands b = g, g + G, ... of d->rowBand rows (rtc.h) */
static RtcRenderDesc part_desc(const RtcRenderDesc *d, int g, int G)
{
    RtcRenderDesc p = *d;
    const int B = d->rowBand > 1 ? d->rowBand : 1;
    p.rowStart = g * B;
    p.rowStride = G;
    p.rowBand = B;
    return p;
}

/* A part's compact rows (d: its part_desc; `elem` bytes per pixel component -- 1 for Color, 4 for the float
 * accumulator) into their places of a host frame of width d->width: one SDMA rectangle per band size (the full bands as
 * rows of B image rows, pitch rowStride*B rows; then the last, partial band), rtc_copy_rows_d2h_dma */
static int copy_part_to_host(unsigned char *hostFrame, const RtcRenderDesc *d, const void *devRows, size_t elem)
{
    const int rows = rtc_rows_selected(d);
    const int B = d->rowBand > 1 ? d->rowBand : 1;
    const size_t rowBytes = (size_t)d->width * 3 * elem;
    unsigned char *dst = hostFrame + (size_t)d->rowStart * rowBytes;
    const size_t hostPitch = (size_t)d->rowStride * B * rowBytes;
    const int full = rows / B, tail = rows - full * B;
    if (full > 0)
        if (int rc = rtc_copy_rows_d2h_dma(dst, hostPitch, devRows, (size_t)B * rowBytes, (size_t)B * rowBytes, full))
            return rc;
    if (tail > 0)
        return rtc_copy_rows_d2h_dma(dst + (size_t)full * hostPitch, rowBytes,
                                     (const unsigned char *)devRows + (size_t)full * B * rowBytes, rowBytes, rowBytes,
                                     tail);
    return 0;
}

extern "C" int rtc_render_multi(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                                const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int numDevices,
                                Color *outImage, float *outAccum, RtcStats *stats)
{
    const auto t0 = std::chrono::steady_clock::now();
    if (!scene || !cam || !d || !outImage || numDevices <= 0 || d->rowStart != 0 || d->rowStride != 1 ||
        d->width <= 0 || d->height <= 0 || d->rowBand < 0 || d->rowBand > 64 || (d->rowBand & (d->rowBand - 1)) != 0)
        return rtc_fail(RTC_EINVAL, "rtc_render_multi: bad argument (full frames only; rowBand: the bands the devices "
                                    "interleave, 0/1 or a power of two <= 64)");
    int n = 0;
    if (int rc = rtc_device_count(&n))
        return rc;
    if (numDevices > n)
        return rtc_fail(RTC_EINVAL, "rtc_render_multi: %d devices requested, %d present", numDevices, n);
    g_multiInfo = MultiInfo{};
    g_multiInfo.devices = numDevices;
    if (d->flags & RTC_F_HOST_ROWS) {
        g_multiInfo.path = 2;
        return rtc_render_multi_host_rows(tris, triCount, spheres, sphereCount, scene, cam, d, numDevices, outImage,
                                          outAccum, stats, t0);
    }
    const Rccl &R = rccl();
    if (!R.ok)
        return rtc_fail(RTC_ENODEV, "rtc_render_multi: RCCL (librccl.so.1) could not be loaded: %s", dlerror());
    RtcDeviceGuard guard(-1);
    const int G = numDevices, W = d->width, H = d->height;
    const RtcRenderDesc d0 = part_desc(d, 0, G);
    const int rowsPer = rtc_rows_selected(&d0); /* every part padded to part 0's row count (the largest) for the gather */
    const size_t partPx = (size_t)rowsPer * (size_t)W;

    /* one communicator per device (single-process clique) */
    std::vector<int> devs(G);
    for (int g = 0; g < G; ++g)
        devs[g] = g;
    std::vector<ncclComm_t> comms(G, nullptr);
    NCCL_TRY(R.commInitAll(comms.data(), G, devs.data()));
    struct CommGuard {
        const Rccl &R;
        std::vector<ncclComm_t> &c;
        ~CommGuard()
        {
            for (ncclComm_t x : c)
                if (x)
                    (void)R.commDestroy(x);
        }
    } commGuard{R, comms};
    g_multiInfo.path = 1;
    for (int g = 0; g < G; ++g) { /* the size of the clique as each communicator sees it (-1: not reported) */
        int c = -1;
        if (!R.commCount || R.commCount(comms[g], &c) != ncclSuccess)
            c = -1;
        g_multiInfo.commRanks.push_back(c);
    }

    /* device 0 also holds the gathered parts and the re-interleaved frame.  Declared before the parts (destroyed
     * after them): the parts' guard synchronises every stream first, so no gather or copy still in flight on an
     * error return touches freed memory. */
    DevBuf<unsigned char> gathered, frame;
    DevBuf<float> gatheredAcc, frameAcc;
    PinnedBuf hColors;
    struct Part {
        RtcDeviceScene *s = nullptr;
        hipStream_t st = nullptr;
        DevBuf<unsigned char> col;
        DevBuf<float> acc;
        DevBuf<unsigned long long> seg;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        int rows = 0;
    };
    std::vector<Part> parts(G);
    const float share = rtc_upload_hit_share(tris, triCount); /* the scheduling hint, estimated once for every device */
    Events evs;
    struct PartsGuard {
        std::vector<Part> &p;
        ~PartsGuard()
        {
            for (size_t g = 0; g < p.size(); ++g) {
                RtcDeviceGuard dg((int)g);
                if (p[g].st)
                    (void)hipStreamSynchronize(p[g].st), (void)hipStreamDestroy(p[g].st);
                rtc_scene_release(p[g].s);
            }
        }
    } partsGuard{parts};
    hipEvent_t eFrame = nullptr;
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        const RtcRenderDesc dg_desc = part_desc(d, g, G);
        p.rows = rtc_rows_selected(&dg_desc);
        if (int rc = rtc_scene_upload_with_share(tris, triCount, spheres, sphereCount, g, share, &p.s))
            return rc;
        HIP_TRY(hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking));
        HIP_TRY(p.col.alloc(partPx * 3, g));
        HIP_TRY(hipMemset(p.col.p, 0, partPx * 3));
        if (outAccum) {
            HIP_TRY(p.acc.alloc(partPx * 3 * sizeof(float), g));
            HIP_TRY(hipMemset(p.acc.p, 0, partPx * 3 * sizeof(float)));
        }
        HIP_TRY(p.seg.alloc(kSegBytes, g));
        HIP_TRY(hipMemset(p.seg.p, 0, kSegBytes));
        HIP_TRY(evs.make(&p.e0));
        HIP_TRY(evs.make(&p.e1));
        if (g == 0) {
            HIP_TRY(gathered.alloc(partPx * 3 * G, 0));
            HIP_TRY(frame.alloc((size_t)W * H * 3, 0));
            if (outAccum) {
                HIP_TRY(gatheredAcc.alloc(partPx * 3 * sizeof(float) * G, 0));
                HIP_TRY(frameAcc.alloc((size_t)W * H * 3 * sizeof(float), 0));
            }
            HIP_TRY(hColors.alloc((size_t)W * H * 3));
            HIP_TRY(evs.make(&eFrame));
        }
    }
    for (int g = 0; g < G; ++g) { /* uploads and memsets done everywhere before the frame starts */
        RtcDeviceGuard dg(g);
        HIP_TRY(hipDeviceSynchronize());
    }

    /* ---- the frame: render every part, gather to device 0 over RCCL, re-interleave, D2H ---- */
    const auto f0 = std::chrono::steady_clock::now();
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        const RtcRenderDesc dg_desc = part_desc(d, g, G);
        HIP_TRY(hipEventRecord(p.e0, p.st));
        if (int rc = rtc_render_rows_async(p.s, scene, cam, &dg_desc, p.col.p, p.acc.p, p.seg.p, p.st))
            return rc;
        HIP_TRY(hipEventRecord(p.e1, p.st));
    }
    NCCL_TRY(R.groupStart());
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        ncclResult_t r = R.gather(p.col.p, g == 0 ? gathered.p : nullptr, partPx * 3, ncclUint8, 0, comms[g], p.st);
        if (r == ncclSuccess && outAccum)
            r = R.gather(p.acc.p, g == 0 ? gatheredAcc.p : nullptr, partPx * 3, ncclFloat32, 0, comms[g], p.st);
        if (r != ncclSuccess) {
            (void)R.groupEnd();
            return rtc_fail((int)r, "ncclGather (device %d): %s", g, R.errorString(r));
        }
    }
    NCCL_TRY(R.groupEnd());
    {
        RtcDeviceGuard dg(0);
        hipStream_t st0 = parts[0].st;
        if (int rc = rtc_deinterleave_bands_async(gathered.p, G, rowsPer, W, H, d0.rowBand, frame.p, st0))
            return rc;
        HIP_TRY(hipMemcpyAsync(hColors.p, frame.p, (size_t)W * H * 3, hipMemcpyDeviceToHost, st0));
        HIP_TRY(hipEventRecord(eFrame, st0));
        HIP_TRY(hipEventSynchronize(eFrame));
    }
    /* the frame time on the host clock: from before the first device's launch until Color[] is on the host (the
     * devices' events cannot be compared across devices) */
    const double frameMs = ms_since(f0);
    if (outAccum) { /* a float row is 4x the bytes of a Color row: re-interleave it as 4W "pixels" */
        RtcDeviceGuard dg(0);
        if (int rc = rtc_deinterleave_bands_async(gatheredAcc.p, G, rowsPer, 4 * W, H, d0.rowBand, frameAcc.p, parts[0].st))
            return rc;
    }
    double renderMs = 0.0;
    unsigned long long seg[RTC_SEGMENT_COUNTERS] = {0};
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        HIP_TRY(hipStreamSynchronize(p.st));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.e0, p.e1));
        renderMs = ms > renderMs ? ms : renderMs;
        unsigned long long sg[RTC_SEGMENT_COUNTERS];
        HIP_TRY(hipMemcpy(sg, p.seg.p, kSegBytes, hipMemcpyDeviceToHost));
        for (int k = 0; k < RTC_SEGMENT_COUNTERS; ++k)
            seg[k] += sg[k];
    }
    memcpy(outImage, hColors.p, (size_t)W * H * 3);
    if (outAccum) {
        RtcDeviceGuard dg(0);
        HIP_TRY(hipMemcpy(outAccum, frameAcc.p, (size_t)W * H * 3 * sizeof(float), hipMemcpyDeviceToHost));
    }
    fill_stats(stats, renderMs, frameMs, seg, d, (size_t)W * H, t0);
    return 0;
}

extern "C" int rtc_last_multi_info(int *path, int *devices, int *commRanks, int maxComms)
{
    if (path)
        *path = g_multiInfo.path;
    if (devices)
        *devices = g_multiInfo.devices;
    const int n = (int)g_multiInfo.commRanks.size();
    for (int i = 0; commRanks && i < n && i < maxComms; ++i)
        commRanks[i] = g_multiInfo.commRanks[(size_t)i];
    return n;
}

/* RTC_F_HOST_ROWS: no gather -- each device copies its compact rows straight into their places of the pinned host
 * frame (rtc_copy_rows_d2h_dma: host pitch G*W*3), over its own PCIe link, concurrently; the reference's threads
 * likewise write their rows into the shared image (main.c:84, :285-302). */
int rtc_render_multi_host_rows(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                               const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int G,
                               Color *outImage, float *outAccum, RtcStats *stats, std::chrono::steady_clock::time_point t0)
{
    RtcDeviceGuard guard(-1);
    const int W = d->width, H = d->height;
    const RtcRenderDesc d0 = part_desc(d, 0, G);
    const int rowsPer = rtc_rows_selected(&d0);
    const size_t partPx = (size_t)rowsPer * (size_t)W;
    PinnedBuf hColors, hAccum; /* before the parts: destroyed after their streams are synchronised */
    HIP_TRY(hColors.alloc((size_t)W * H * 3));
    if (outAccum)
        HIP_TRY(hAccum.alloc((size_t)W * H * 3 * sizeof(float)));
    struct Part {
        RtcDeviceScene *s = nullptr;
        hipStream_t st = nullptr;
        DevBuf<unsigned char> col;
        DevBuf<float> acc;
        DevBuf<unsigned long long> seg;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        int rows = 0;
        int rc = 0;
        std::string err;
    };
    std::vector<Part> parts(G);
    const float share = rtc_upload_hit_share(tris, triCount); /* the scheduling hint, estimated once for every device */
    Events evs;
    struct PartsGuard {
        std::vector<Part> &p;
        ~PartsGuard()
        {
            for (size_t g = 0; g < p.size(); ++g) {
                RtcDeviceGuard dg((int)g);
                if (p[g].st)
                    (void)hipStreamSynchronize(p[g].st), (void)hipStreamDestroy(p[g].st);
                rtc_scene_release(p[g].s);
            }
        }
    } partsGuard{parts};
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        const RtcRenderDesc dg_desc = part_desc(d, g, G);
        p.rows = rtc_rows_selected(&dg_desc);
        if (int rc = rtc_scene_upload_with_share(tris, triCount, spheres, sphereCount, g, share, &p.s))
            return rc;
        HIP_TRY(hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking));
        HIP_TRY(p.col.alloc(partPx * 3 + 16, g));
        if (outAccum)
            HIP_TRY(p.acc.alloc(partPx * 3 * sizeof(float) + 16, g));
        HIP_TRY(p.seg.alloc(kSegBytes, g));
        HIP_TRY(hipMemset(p.seg.p, 0, kSegBytes));
        HIP_TRY(evs.make(&p.e0));
        HIP_TRY(evs.make(&p.e1));
        HIP_TRY(hipDeviceSynchronize());
    }
    const auto f0 = std::chrono::steady_clock::now();
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        const RtcRenderDesc dg_desc = part_desc(d, g, G);
        HIP_TRY(hipEventRecord(p.e0, p.st));
        if (int rc = rtc_render_rows_async(p.s, scene, cam, &dg_desc, p.col.p, p.acc.p, p.seg.p, p.st))
            return rc;
        HIP_TRY(hipEventRecord(p.e1, p.st));
    }
    /* one host thread per device: wait for its rows, copy them into the frame (SDMA, own link) */
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g] {
            Part &p = parts[g];
            RtcDeviceGuard dg(g);
            hipError_t e = hipEventSynchronize(p.e1);
            if (e != hipSuccess) {
                p.rc = rtc_fail(-(int)e, "rtc_render_multi: device %d: %s", g, hipGetErrorString(e));
            } else {
                const RtcRenderDesc pd = part_desc(d, g, G);
                p.rc = copy_part_to_host((unsigned char *)hColors.p, &pd, p.col.p, 1);
            }
            if (p.rc)
                p.err = rtc_last_error();
        });
    for (std::thread &t : th)
        t.join();
    const double frameMs = ms_since(f0);
    for (int g = 0; g < G; ++g)
        if (parts[g].rc)
            return rtc_fail(parts[g].rc, "%s", parts[g].err.c_str());
    double renderMs = 0.0;
    unsigned long long seg[RTC_SEGMENT_COUNTERS] = {0};
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.e0, p.e1));
        renderMs = ms > renderMs ? ms : renderMs;
        unsigned long long sg[RTC_SEGMENT_COUNTERS];
        HIP_TRY(hipMemcpy(sg, p.seg.p, kSegBytes, hipMemcpyDeviceToHost));
        for (int k = 0; k < RTC_SEGMENT_COUNTERS; ++k)
            seg[k] += sg[k];
        if (outAccum) {
            const RtcRenderDesc pd = part_desc(d, g, G);
            if (int rc = copy_part_to_host((unsigned char *)hAccum.p, &pd, p.acc.p, sizeof(float)))
                return rc;
        }
    }
    memcpy(outImage, hColors.p, (size_t)W * H * 3);
    if (outAccum)
        memcpy(outAccum, hAccum.p, (size_t)W * H * 3 * sizeof(float));
    fill_stats(stats, renderMs, frameMs, seg, d, (size_t)W * H, t0);
    return 0;
}

/* ---- D2H through the copy engines ------------------------------------------------------------------------
 * The HIP runtime copies device memory into pinned host memory with a blit kernel (one workgroup per CU); while
 * render kernels run, those PCIe writes from the shader cores cost the render ~0.1 ms per 1080p frame, even from a
 * handful of workgroups, whereas the SDMA engines' copy costs it ~0.01 ms.  The copies below drive the SDMA engines
 * through the HSA runtime HIP itself runs on, blocking, for a caller thread that pipelines frame copies behind the
 * renders.  The destination is page-locked host memory: hipHostMalloc'd (HSA pointer type HSA) or registered
 * (hipHostRegister / rtc_host_register: type LOCKED, reached by the GPU at its agent address).  The host side of the
 * copy is the CPU agent nearest the source GPU (HSA_AMD_AGENT_INFO_NEAREST_CPU), so a GPU on the second socket does
 * not stage through the first. */
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <mutex>

namespace {
struct DmaAgents {
    std::vector<hsa_agent_t> cpu;
    bool ok = false;
};
DmaAgents &dma_agents()
{
    static DmaAgents a;
    static std::once_flag once;
    std::call_once(once, [] {
        if (hsa_init() != HSA_STATUS_SUCCESS) /* reference-counted: HIP has initialised it already */
            return;
        hsa_iterate_agents(
            [](hsa_agent_t ag, void *p) -> hsa_status_t {
                hsa_device_type_t t;
                if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU)
                    static_cast<DmaAgents *>(p)->cpu.push_back(ag);
                return HSA_STATUS_SUCCESS;
            },
            &a);
        a.ok = !a.cpu.empty();
    });
    return a;
}

/* ranges page-locked by rtc_host_register: host base -> (bytes, the agents' address).  The HSA runtime's pointer
 * info does not report these host addresses, so the copies look them up here. */
struct LockedRange {
    size_t bytes;
    void *agent;
};
std::mutex g_lockedMu;
std::map<uintptr_t, LockedRange> g_locked;

/* the agents' address of [p, p + span) inside one registered range, or null */
void *locked_agent_address(const void *p, size_t span)
{
    std::lock_guard<std::mutex> lk(g_lockedMu);
    const uintptr_t a = (uintptr_t)p;
    auto it = g_locked.upper_bound(a);
    if (it == g_locked.begin())
        return nullptr;
    --it;
    const uintptr_t off = a - it->first;
    if (off + span > it->second.bytes)
        return nullptr;
    return (char *)it->second.agent + off;
}

/* one completion signal per calling thread, destroyed with the thread */
struct DmaSignal {
    hsa_signal_t s{0};
    ~DmaSignal()
    {
        if (s.handle)
            (void)hsa_signal_destroy(s);
    }
};

/* Copies that did not complete within the wait limit (dma_wait): the engine may still read [srcLo, srcHi) and write
 * [dstLo, dstHi) and decrement `sig`.  They stay listed -- their signal neither reused nor destroyed -- until the signal
 * shows the copy ended (rtc_dma_pending reaps them); rtc_host_unregister refuses a range one of them may still write.
 * `simulated` entries (rtc_dma_debug_inflight, CPU tests of this bookkeeping) have no signal. */
struct InflightCopy {
    uintptr_t dstLo, dstHi, srcLo, srcHi;
    hsa_signal_t sig;
};
std::mutex g_inflightMu;
std::vector<InflightCopy> g_inflight;

/* copies still pending whose destination or source overlaps [lo, hi); finished ones are reaped */
int inflight_overlapping(uintptr_t lo, uintptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_inflightMu);
    int n = 0;
    for (size_t i = 0; i < g_inflight.size();) {
        InflightCopy &c = g_inflight[i];
        if (c.sig.handle && hsa_signal_load_scacquire(c.sig) < 1) { /* completed (0) or failed (< 0): engine done */
            (void)hsa_signal_destroy(c.sig);
            g_inflight.erase(g_inflight.begin() + (ptrdiff_t)i);
            continue;
        }
        n += (c.dstLo < hi && lo < c.dstHi) || (c.srcLo < hi && lo < c.srcHi);
        ++i;
    }
    return n;
}

/* wait until the thread's copy signal drops below 1; RTC_EIO when the copy reports an error (negative value).  After
 * the wait limit (20 s, RTC_DMA_TIMEOUT_MS) a faulted or lost copy must not hang the caller, but the engine may still
 * write: the copy is listed in flight with its signal (the thread takes a fresh one for its next copy) and
 * RTC_ETIMEDOUT tells the caller not to free, reuse or unregister dst / src until rtc_dma_pending says it ended. */
int dma_wait(hsa_signal_t &sig, const void *dst, size_t dstBytes, const void *src, size_t srcBytes, const char *what)
{
    static const double limitMs = [] {
        const char *e = getenv("RTC_DMA_TIMEOUT_MS");
        return e && atof(e) > 0.0 ? atof(e) : 20000.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 1000000,
                                                                HSA_WAIT_STATE_BLOCKED);
        if (v == 0)
            return 0;
        if (v < 0)
            return rtc_fail(RTC_EIO, "%s: the copy engine reported an error (signal %lld)", what, (long long)v);
        if (ms_since(t0) > limitMs) {
            {
                std::lock_guard<std::mutex> lk(g_inflightMu);
                g_inflight.push_back(InflightCopy{(uintptr_t)dst, (uintptr_t)dst + dstBytes, (uintptr_t)src,
                                                  (uintptr_t)src + srcBytes, sig});
            }
            sig.handle = 0; /* owned by the in-flight list now */
            return rtc_fail(RTC_ETIMEDOUT, "%s: copy not completed after %.0f ms; it may still write its destination "
                                           "(rtc_dma_pending)", what, limitMs);
        }
    }
}

/* The source's GPU agent, the destination's GPU-visible address and the copy's CPU agent.  hostDst..+span must lie
 * in one page-locked allocation. */
int dma_endpoints(void *hostDst, size_t span, const void *devSrc, const char *what, hsa_agent_t &gpu, void *&dstAgent,
                  hsa_agent_t &cpu)
{
    DmaAgents &a = dma_agents();
    if (!a.ok)
        return rtc_fail(RTC_ENODEV, "%s: no HSA CPU agent", what);
    hsa_amd_pointer_info_t src{}, dst{};
    src.size = sizeof(src);
    dst.size = sizeof(dst);
    if (hsa_amd_pointer_info(devSrc, &src, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        src.type != HSA_EXT_POINTER_TYPE_HSA)
        return rtc_fail(RTC_EINVAL, "%s: source is not device memory", what);
    const hsa_status_t pi = hsa_amd_pointer_info(hostDst, &dst, nullptr, nullptr, nullptr);
    if (pi == HSA_STATUS_SUCCESS && (dst.type == HSA_EXT_POINTER_TYPE_HSA || dst.type == HSA_EXT_POINTER_TYPE_LOCKED)) {
        const size_t off = (size_t)((const char *)hostDst - (const char *)dst.hostBaseAddress);
        /* hipHostMalloc: the same address on every agent; registered (locked) memory: the GPU reaches it at its
         * agent address */
        dstAgent = dst.type == HSA_EXT_POINTER_TYPE_HSA ? hostDst : (void *)((char *)dst.agentBaseAddress + off);
        if (off + span > dst.sizeInBytes)
            return rtc_fail(RTC_EINVAL, "%s: destination range leaves its page-locked allocation", what);
    } else if (!(dstAgent = locked_agent_address(hostDst, span))) {
        return rtc_fail(RTC_EINVAL, "%s: destination is not page-locked host memory (HSA pointer type %d)", what,
                        pi == HSA_STATUS_SUCCESS ? (int)dst.type : -1);
    }
    gpu = src.agentOwner;
    cpu = a.cpu[0];
    hsa_agent_t near{0};
    if (hsa_agent_get_info(gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &near) == HSA_STATUS_SUCCESS &&
        near.handle)
        cpu = near;
    return 0;
}
} // namespace

extern "C" int rtc_copy_d2h_dma(void *hostDst, const void *devSrc, size_t bytes)
{
    if ((!hostDst || !devSrc) && bytes)
        return rtc_fail(RTC_EINVAL, "rtc_copy_d2h_dma: null pointer");
    if (bytes == 0)
        return 0;
    hsa_agent_t gpu, cpu;
    void *dst = nullptr;
    if (int rc = dma_endpoints(hostDst, bytes, devSrc, "rtc_copy_d2h_dma", gpu, dst, cpu))
        return rc;
    thread_local DmaSignal sig;
    if (!sig.s.handle && hsa_signal_create(1, 0, nullptr, &sig.s) != HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_ENOMEM, "rtc_copy_d2h_dma: hsa_signal_create failed");
    hsa_signal_store_screlease(sig.s, 1);
    if (hsa_amd_memory_async_copy(dst, cpu, devSrc, gpu, bytes, 0, nullptr, sig.s) != HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_EIO, "rtc_copy_d2h_dma: hsa_amd_memory_async_copy failed");
    return dma_wait(sig.s, hostDst, bytes, devSrc, bytes, "rtc_copy_d2h_dma");
}

extern "C" int rtc_copy_rows_d2h_dma(void *hostDst, size_t hostPitch, const void *devSrc, size_t srcPitch,
                                     size_t rowBytes, int rows)
{
    if (rows < 0 || (rows > 0 && rowBytes > 0 && (!hostDst || !devSrc)) || (rows > 1 && (hostPitch < rowBytes ||
                                                                                         srcPitch < rowBytes)))
        return rtc_fail(RTC_EINVAL, "rtc_copy_rows_d2h_dma: bad argument");
    if (rows == 0 || rowBytes == 0)
        return 0;
    const size_t span = (size_t)(rows - 1) * hostPitch + rowBytes, srcSpan = (size_t)(rows - 1) * srcPitch + rowBytes;
    hsa_agent_t gpu, cpu;
    void *dst = nullptr;
    if (int rc = dma_endpoints(hostDst, span, devSrc, "rtc_copy_rows_d2h_dma", gpu, dst, cpu))
        return rc;
    thread_local DmaSignal sig;
    if (!sig.s.handle && hsa_signal_create(1, 0, nullptr, &sig.s) != HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_ENOMEM, "rtc_copy_rows_d2h_dma: hsa_signal_create failed");
    const bool dense = rows == 1 || (hostPitch == rowBytes && srcPitch == rowBytes);
    const bool aligned4 = (((uintptr_t)dst | (uintptr_t)devSrc | hostPitch | srcPitch | rowBytes) & 3u) == 0;
    if (dense) {
        hsa_signal_store_screlease(sig.s, 1);
        if (hsa_amd_memory_async_copy(dst, cpu, devSrc, gpu, (size_t)rows * rowBytes, 0, nullptr, sig.s) !=
            HSA_STATUS_SUCCESS)
            return rtc_fail(RTC_EIO, "rtc_copy_rows_d2h_dma: hsa_amd_memory_async_copy failed");
    } else if (aligned4) {
        /* one SDMA sub-window copy: x in bytes, y in rows */
        hsa_pitched_ptr_t d{dst, hostPitch, hostPitch * (size_t)rows}, sp{const_cast<void *>(devSrc), srcPitch,
                                                                          srcPitch * (size_t)rows};
        const hsa_dim3_t zero{0, 0, 0}, range{(uint32_t)rowBytes, (uint32_t)rows, 1};
        hsa_signal_store_screlease(sig.s, 1);
        if (hsa_amd_memory_async_copy_rect(&d, &zero, &sp, &zero, &range, gpu, hsaDeviceToHost, 0, nullptr, sig.s) !=
            HSA_STATUS_SUCCESS)
            return rtc_fail(RTC_EIO, "rtc_copy_rows_d2h_dma: hsa_amd_memory_async_copy_rect failed");
    } else {
        /* rows that are not 4-byte aligned: one linear SDMA copy per row, all on one signal */
        hsa_signal_store_screlease(sig.s, rows);
        for (int r = 0; r < rows; ++r)
            if (hsa_amd_memory_async_copy((char *)dst + (size_t)r * hostPitch, cpu, (const char *)devSrc + (size_t)r * srcPitch,
                                          gpu, rowBytes, 0, nullptr, sig.s) != HSA_STATUS_SUCCESS) {
                hsa_signal_subtract_screlease(sig.s, rows - r); /* the copies not issued */
                /* drain the copies already issued; if that wait timed out they may still write hostDst: report
                 * RTC_ETIMEDOUT (rtc_dma_pending lists them), not RTC_EIO */
                if (int wrc = dma_wait(sig.s, hostDst, span, devSrc, srcSpan, "rtc_copy_rows_d2h_dma"))
                    return wrc;
                return rtc_fail(RTC_EIO, "rtc_copy_rows_d2h_dma: hsa_amd_memory_async_copy failed (row %d)", r);
            }
    }
    return dma_wait(sig.s, hostDst, span, devSrc, srcSpan, "rtc_copy_rows_d2h_dma");
}

/* Page-locked through the HSA runtime itself (hsa_amd_memory_lock for every agent), so the range has the LOCKED
 * pointer type rtc_copy_*_d2h_dma resolve to the GPU's agent address, whatever backs it (e.g. a shared-memory file
 * mapping every rank of a node maps). */
extern "C" int rtc_host_register(void *p, size_t bytes)
{
    if (!p || !bytes)
        return rtc_fail(RTC_EINVAL, "rtc_host_register: empty range");
    if (!dma_agents().ok)
        return rtc_fail(RTC_ENODEV, "rtc_host_register: no HSA runtime");
    void *agentPtr = nullptr;
    if (hsa_amd_memory_lock(p, bytes, nullptr, 0, &agentPtr) != HSA_STATUS_SUCCESS || !agentPtr)
        return rtc_fail(RTC_EIO, "rtc_host_register: hsa_amd_memory_lock failed");
    std::lock_guard<std::mutex> lk(g_lockedMu);
    g_locked[(uintptr_t)p] = LockedRange{bytes, agentPtr};
    return 0;
}

extern "C" int rtc_host_unregister(void *p)
{
    if (!p)
        return rtc_fail(RTC_EINVAL, "rtc_host_unregister: null pointer");
    size_t bytes = 1;
    {
        std::lock_guard<std::mutex> lk(g_lockedMu);
        auto it = g_locked.find((uintptr_t)p);
        if (it != g_locked.end())
            bytes = it->second.bytes;
    }
    if (const int n = inflight_overlapping((uintptr_t)p, (uintptr_t)p + bytes))
        return rtc_fail(RTC_EBUSY, "rtc_host_unregister: %d timed-out copies may still write this range", n);
    {
        std::lock_guard<std::mutex> lk(g_lockedMu);
        g_locked.erase((uintptr_t)p);
    }
    if (hsa_amd_memory_unlock(p) != HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_EIO, "rtc_host_unregister: hsa_amd_memory_unlock failed");
    return 0;
}

extern "C" int rtc_dma_pending(const void *p, size_t bytes)
{
    if (!p && bytes)
        return rtc_fail(RTC_EINVAL, "rtc_dma_pending: null pointer");
    return p ? inflight_overlapping((uintptr_t)p, (uintptr_t)p + (bytes ? bytes : 1))
             : inflight_overlapping(0, ~(uintptr_t)0);
}

extern "C" int rtc_dma_debug_inflight(void *p, size_t bytes, int pending)
{
    if (!p || !bytes)
        return rtc_fail(RTC_EINVAL, "rtc_dma_debug_inflight: empty range");
    std::lock_guard<std::mutex> lk(g_inflightMu);
    if (pending) {
        g_inflight.push_back(InflightCopy{(uintptr_t)p, (uintptr_t)p + bytes, 0, 0, hsa_signal_t{0}});
        return 0;
    }
    for (size_t i = 0; i < g_inflight.size(); ++i)
        if (!g_inflight[i].sig.handle && g_inflight[i].dstLo == (uintptr_t)p && g_inflight[i].dstHi == (uintptr_t)p + bytes) {
            g_inflight.erase(g_inflight.begin() + (ptrdiff_t)i);
            return 0;
        }
    return rtc_fail(RTC_EINVAL, "rtc_dma_debug_inflight: no simulated copy for this range");
}

/* ---- pipelined frames (the host frame loop) -------------------------------------------------------------------
 * A frame sequence on one device, driven from native code so the per-frame host cost is the launch enqueue alone:
 * frame k renders the rows of d (RTC_F_OVERLAP: its preparation overlaps frame k-1's sky pass) into devRows[k %
 * nbuf]; a copy thread waits for the frame's event and moves its rows into hostRows[k % nbuf] (pitch hostPitch between
 * consecutive rows -- or bands of d->rowBand rows: a rank's rows y = rowStart + j*rowStride land in the interleaved host
 * frame when hostRows points at row rowStart and hostPitch = rowStride * rowBand * width * 3) on the SDMA engines; buffer b is rendered into again once its copy has
 * finished.  The reference's equivalent is main.c:285-305: the threads write their rows into the shared image, which
 * stbi_write_bmp then reads. */

extern "C" int rtc_frame_loop_cameras(RtcDeviceScene *s, const Scene *scene, const RtcCamera *cams, int ncams,
                                      const RtcRenderDesc *d, void *const *devRows, void *const *hostRows,
                                      size_t hostPitch, int nbuf, int frames, void *stream, RtcLoopStats *stats)
{
    if (!s || !scene || !cams || ncams <= 0 || !d || !devRows || !hostRows || nbuf <= 0 || nbuf > 16 || frames < 0)
        return rtc_fail(RTC_EINVAL, "rtc_frame_loop: bad argument");
    for (int b = 0; b < nbuf; ++b)
        if (!devRows[b] || !hostRows[b])
            return rtc_fail(RTC_EINVAL, "rtc_frame_loop: null buffer %d", b);
    const int rows = rtc_rows_selected(d);
    const size_t rowBytes = (size_t)(d->width > 0 ? d->width : 0) * 3;
    const int B = d->rowBand > 1 ? d->rowBand : 1;
    if (rows > B && hostPitch < (size_t)B * rowBytes)
        return rtc_fail(RTC_EINVAL, "rtc_frame_loop: host pitch %zu < band bytes %zu", hostPitch, (size_t)B * rowBytes);
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    RtcRenderDesc dd = *d;
    dd.flags |= RTC_F_OVERLAP;
    Events evs;
    std::vector<hipEvent_t> ready(nbuf);
    for (int b = 0; b < nbuf; ++b) {
        HIP_TRY(hipEventCreateWithFlags(&ready[b], hipEventDisableTiming));
        evs.ev.push_back(ready[b]);
    }
    std::mutex m;
    std::condition_variable cv;
    std::deque<int> jobs;
    std::vector<char> busy(nbuf, 0);
    std::vector<double> copyMs;
    copyMs.reserve(frames);
    int err = 0;
    std::string errMsg;
    bool done = false;
    std::thread copier([&] {
        RtcDeviceGuard g(device);
        for (;;) {
            int b;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return done || !jobs.empty(); });
                if (jobs.empty())
                    return;
                b = jobs.front();
                jobs.pop_front();
            }
            int rc = 0;
            double ms = 0.0;
            const hipError_t e = hipEventSynchronize(ready[b]);
            if (e != hipSuccess) {
                rc = rtc_fail(-(int)e, "rtc_frame_loop: frame event: %s", hipGetErrorString(e));
            } else {
                const auto c0 = std::chrono::steady_clock::now();
                /* bands of B rows (d->rowBand): the full bands as rows of B image rows at the band pitch, then the
                 * last, partial band (single rows: B = 1, one rectangle) */
                const int full = rows / B, tail = rows - full * B;
                rc = full > 0 ? rtc_copy_rows_d2h_dma(hostRows[b], hostPitch, devRows[b], B * rowBytes, B * rowBytes, full)
                              : 0;
                if (!rc && tail > 0)
                    rc = rtc_copy_rows_d2h_dma((unsigned char *)hostRows[b] + (size_t)full * hostPitch, rowBytes,
                                               (const unsigned char *)devRows[b] + (size_t)full * B * rowBytes, rowBytes,
                                               rowBytes, tail);
                ms = ms_since(c0);
            }
            std::lock_guard<std::mutex> lk(m);
            if (rc && !err) {
                err = rc;
                errMsg = rtc_last_error();
            }
            copyMs.push_back(ms);
            busy[b] = 0;
            cv.notify_all();
        }
    });
    const auto t0 = std::chrono::steady_clock::now();
    double enqueueMs = 0.0;
    int rc = 0;
    for (int k = 0; k < frames && !rc; ++k) {
        const int b = k % nbuf;
        {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return !busy[b] || err; });
            if (err)
                break;
            busy[b] = 1;
        }
        const auto e0 = std::chrono::steady_clock::now();
        rc = rtc_scene_set_frame_event(s, ready[b]);
        if (!rc)
            rc = rtc_render_rows_async(s, scene, &cams[k % ncams], &dd, devRows[b], nullptr, nullptr, stream);
        enqueueMs += ms_since(e0);
        if (!rc) {
            std::lock_guard<std::mutex> lk(m);
            jobs.push_back(b);
            cv.notify_all();
        }
    }
    {
        std::lock_guard<std::mutex> lk(m);
        done = true;
        cv.notify_all();
    }
    copier.join();
    (void)rtc_scene_set_frame_event(s, nullptr); /* never leave ready[] armed: it is destroyed on return */
    const double wall = ms_since(t0);
    if (!rc && err)
        rc = rtc_fail(err, "%s", errMsg.c_str());
    if (!rc) { /* the frames are on the host; the scene's unjoined sky pass of the last frame has finished too */
        const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
        if (e != hipSuccess)
            rc = rtc_fail(-(int)e, "rtc_frame_loop: %s", hipGetErrorString(e));
    }
    if (stats) {
        std::sort(copyMs.begin(), copyMs.end());
        stats->wallMs = wall;
        stats->frames = frames;
        stats->enqueueMs = enqueueMs;
        stats->copyMsMedian = copyMs.empty() ? 0.0 : copyMs[copyMs.size() / 2];
        stats->copyMsMax = copyMs.empty() ? 0.0 : copyMs.back();
    }
    return rc;
}

extern "C" int rtc_frame_loop(RtcDeviceScene *s, const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d,
                              void *const *devRows, void *const *hostRows, size_t hostPitch, int nbuf, int frames,
                              void *stream, RtcLoopStats *stats)
{
    if (!cam)
        return rtc_fail(RTC_EINVAL, "rtc_frame_loop: bad argument");
    return rtc_frame_loop_cameras(s, scene, cam, 1, d, devRows, hostRows, hostPitch, nbuf, frames, stream, stats);
}

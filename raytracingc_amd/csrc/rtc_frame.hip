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

#include <chrono>
#include <cstring>
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
    bool ok = false;
};

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

extern "C" int rtc_render_multi(const Triangle *tris, int triCount, const Sphere *spheres, int sphereCount,
                                const Scene *scene, const RtcCamera *cam, const RtcRenderDesc *d, int numDevices,
                                Color *outImage, float *outAccum, RtcStats *stats)
{
    const auto t0 = std::chrono::steady_clock::now();
    if (!scene || !cam || !d || !outImage || numDevices <= 0 || d->rowStart != 0 || d->rowStride != 1 ||
        d->width <= 0 || d->height <= 0)
        return rtc_fail(RTC_EINVAL, "rtc_render_multi: bad argument (full frames only)");
    int n = 0;
    if (int rc = rtc_device_count(&n))
        return rc;
    if (numDevices > n)
        return rtc_fail(RTC_EINVAL, "rtc_render_multi: %d devices requested, %d present", numDevices, n);
    const Rccl &R = rccl();
    if (!R.ok)
        return rtc_fail(RTC_ENODEV, "rtc_render_multi: RCCL (librccl.so.1) could not be loaded: %s", dlerror());
    RtcDeviceGuard guard(-1);
    const int G = numDevices, W = d->width, H = d->height;
    const int rowsPer = (H + G - 1) / G; /* every part padded to rank 0's row count for the gather */
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
    /* device 0 also holds the gathered parts, the re-interleaved frame and the events around the frame */
    DevBuf<unsigned char> gathered, frame;
    DevBuf<float> gatheredAcc, frameAcc;
    PinnedBuf hColors;
    hipEvent_t eFrame = nullptr;
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        RtcRenderDesc dg_desc = *d;
        dg_desc.rowStart = g;
        dg_desc.rowStride = G;
        p.rows = rtc_rows_selected(&dg_desc);
        if (int rc = rtc_scene_upload(tris, triCount, spheres, sphereCount, g, &p.s))
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
    for (int g = 0; g < G; ++g) {
        Part &p = parts[g];
        RtcDeviceGuard dg(g);
        RtcRenderDesc dg_desc = *d;
        dg_desc.rowStart = g;
        dg_desc.rowStride = G;
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
        if (int rc = rtc_deinterleave_async(gathered.p, G, rowsPer, W, H, frame.p, st0))
            return rc;
        HIP_TRY(hipMemcpyAsync(hColors.p, frame.p, (size_t)W * H * 3, hipMemcpyDeviceToHost, st0));
        HIP_TRY(hipEventRecord(eFrame, st0));
        if (outAccum) /* a float row is 4x the bytes of a Color row: re-interleave it as 4W "pixels" */
            if (int rc = rtc_deinterleave_async(gatheredAcc.p, G, rowsPer, 4 * W, H, frameAcc.p, st0))
                return rc;
        HIP_TRY(hipEventSynchronize(eFrame));
    }
    float frameMs = 0.f;
    {
        RtcDeviceGuard dg(0);
        HIP_TRY(hipEventElapsedTime(&frameMs, parts[0].e0, eFrame));
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

/* ---- D2H through the copy engines ------------------------------------------------------------------------
 * The HIP runtime copies device memory into pinned host memory with a blit kernel (one workgroup per CU); while
 * render kernels run, those PCIe writes from the shader cores cost the render ~0.1 ms per 1080p frame, even
 * from a handful of workgroups (tools/copy_overlap_probe.py), whereas the SDMA engines' copy costs it ~0.01 ms
 * (tools/sdma_overlap_probe.py).  rtc_copy_d2h_dma drives the SDMA engines through the HSA runtime HIP itself
 * runs on: blocking, for a caller thread that pipelines frame copies behind the renders. */
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
} // namespace

extern "C" int rtc_copy_d2h_dma(void *hostDst, const void *devSrc, size_t bytes)
{
    if ((!hostDst || !devSrc) && bytes)
        return rtc_fail(RTC_EINVAL, "rtc_copy_d2h_dma: null pointer");
    if (bytes == 0)
        return 0;
    DmaAgents &a = dma_agents();
    if (!a.ok)
        return rtc_fail(RTC_ENODEV, "rtc_copy_d2h_dma: no HSA CPU agent");
    /* the GPU agent that owns the source, and the destination must be page-locked (hipHostMalloc) memory */
    hsa_amd_pointer_info_t src{}, dst{};
    src.size = sizeof(src);
    dst.size = sizeof(dst);
    if (hsa_amd_pointer_info(devSrc, &src, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        src.type != HSA_EXT_POINTER_TYPE_HSA)
        return rtc_fail(RTC_EINVAL, "rtc_copy_d2h_dma: source is not device memory");
    if (hsa_amd_pointer_info(hostDst, &dst, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        (dst.type != HSA_EXT_POINTER_TYPE_HSA && dst.type != HSA_EXT_POINTER_TYPE_LOCKED))
        return rtc_fail(RTC_EINVAL, "rtc_copy_d2h_dma: destination is not page-locked host memory");
    thread_local hsa_signal_t sig{0};
    if (!sig.handle && hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_ENOMEM, "rtc_copy_d2h_dma: hsa_signal_create failed");
    hsa_signal_store_screlease(sig, 1);
    if (hsa_amd_memory_async_copy(hostDst, a.cpu[0], devSrc, src.agentOwner, bytes, 0, nullptr, sig) !=
        HSA_STATUS_SUCCESS)
        return rtc_fail(RTC_EIO, "rtc_copy_d2h_dma: hsa_amd_memory_async_copy failed");
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    return 0;
}

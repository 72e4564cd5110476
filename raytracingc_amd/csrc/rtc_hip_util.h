/* rtc_hip_util.h -- host-side helpers shared by the HIP translation units of librtc.so (C++ only). */
#pragma once
#include <hip/hip_runtime.h>

#include "rtc_internal.h"

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return rtc_fail(-(int)e_, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                            __LINE__);                                                                 \
    } while (0)

/* Every extern "C" entry point that selects a device restores the caller's current device on return, so
 * a call such as rtc_render(..., device = 1) or rtc_render_multi(N) never moves the process's (or torch's)
 * current device.  `device` < 0 keeps the current one. */
class RtcDeviceGuard {
  public:
    explicit RtcDeviceGuard(int device)
    {
        if (hipGetDevice(&prev_) != hipSuccess)
            prev_ = -1;
        if (device >= 0 && device != prev_)
            ok_ = hipSetDevice(device) == hipSuccess;
    }
    ~RtcDeviceGuard()
    {
        int cur = -1;
        if (prev_ >= 0 && (hipGetDevice(&cur) != hipSuccess || cur != prev_))
            (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }
    RtcDeviceGuard(const RtcDeviceGuard &) = delete;
    RtcDeviceGuard &operator=(const RtcDeviceGuard &) = delete;

  private:
    int prev_ = -1;
    bool ok_ = true;
};

/* rtc_internal.h -- helpers shared by the host (C) and HIP translation units of librtc.so. */
#ifndef RTC_INTERNAL_H
#define RTC_INTERNAL_H

#ifdef __cplusplus
extern "C" {
#endif

/* Record a thread-local error message for rtc_last_error() and return `code`. */
int rtc_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
/* Loader diagnostics (objloader.c prints them with PRINT_LOADING); quiet unless RTC_VERBOSE >= level. */
void rtc_log(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
/* rtc_scene_upload with the scheduling hint bounce_hit_share already known (hitShare >= 0; < 0: estimate it): the
 * multi-device paths estimate it once for every device's upload */
struct Triangle;
struct Sphere;
struct RtcDeviceScene;
float rtc_upload_hit_share(const struct Triangle *tris, int triCount); /* what rtc_scene_upload estimates */
int rtc_scene_upload_with_share(const struct Triangle *tris, int triCount, const struct Sphere *spheres, int sphereCount,
                                int device, float hitShare, struct RtcDeviceScene **out);

#ifdef __cplusplus
}
#endif
#endif

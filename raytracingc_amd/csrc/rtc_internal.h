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

#ifdef __cplusplus
}
#endif
#endif

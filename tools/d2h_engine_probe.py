#!/usr/bin/env python3
"""Which engine carries a 6.2 MB D2H copy into pinned memory (blit kernel or SDMA), by host-allocation kind and
API; run under rocprofv3 --kernel-trace --memory-copy-trace.  Not part of the product."""
import ctypes as C
import os

import torch

hip = C.CDLL("libamdhip64.so")
n = 1920 * 1080 * 3
src = torch.zeros(n, dtype=torch.uint8, device="cuda")
st = torch.cuda.Stream()
print("HSA_ENABLE_SDMA =", os.environ.get("HSA_ENABLE_SDMA"), flush=True)


def timed(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
with torch.cuda.stream(st):
    print("torch pinned copy_ ms", round(timed(lambda: pinned.copy_(src, non_blocking=True)), 4), flush=True)
hostp = C.c_void_p()
for flags, name in ((0x0, "hipHostMalloc default"), (0x2, "hipHostMalloc mapped"), (0x40000000, "hipHostMalloc noncoherent")):
    if hip.hipHostMalloc(C.byref(hostp), C.c_size_t(n), C.c_uint(flags)) != 0:
        print(name, "alloc failed")
        continue
    f = lambda: hip.hipMemcpyAsync(hostp, C.c_void_p(src.data_ptr()), C.c_size_t(n), C.c_int(2), C.c_void_p(st.cuda_stream))
    print(name, "hipMemcpyAsync D2H ms", round(timed(f), 4), flush=True)
    f2 = lambda: hip.hipMemcpyDtoHAsync(hostp, C.c_void_p(src.data_ptr()), C.c_size_t(n), C.c_void_p(st.cuda_stream))
    print(name, "hipMemcpyDtoHAsync ms", round(timed(f2), 4), flush=True)
    hip.hipHostFree(hostp)

# hipMemcpyDeviceToDeviceNoCU (1024): the copy engines (SDMA) instead of a blit kernel, into pinned memory
src.copy_(torch.arange(n, dtype=torch.int64, device="cuda").to(torch.uint8))
torch.cuda.synchronize()
pinned2 = torch.zeros(n, dtype=torch.uint8, pin_memory=True)
f3 = lambda: hip.hipMemcpyAsync(C.c_void_p(pinned2.data_ptr()), C.c_void_p(src.data_ptr()), C.c_size_t(n), C.c_int(1024),
                                C.c_void_p(st.cuda_stream))
rc = f3()
torch.cuda.synchronize()
print("NoCU rc", rc, "equal", bool(torch.equal(pinned2, src.cpu())), flush=True)
if rc == 0:
    print("torch pinned hipMemcpyAsync NoCU ms", round(timed(f3), 4), flush=True)

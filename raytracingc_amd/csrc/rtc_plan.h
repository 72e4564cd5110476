/*
 * rtc_plan.h -- the launch planner of rtc_render_rows_async (pure host code: no HIP, no device memory).
 *
 * One call of rtc_render_rows_async is the reference's render region (main.c:263-304) as a short sequence of kernels on
 * up to four streams: the caller's, two cull streams and the scene's side stream.  Pipelined
 * launches (RTC_F_OVERLAP) are in flight together, so every buffer two of them may touch at once needs either its own
 * copy (a scratch slot, a counter set) or an event between them.  rtc_plan_launch decides all of it from the scene's
 * ordering state and the launch's shape -- the scratch slot and its byte layout, the streams, every event record and
 * wait, which kernels run and which event each one completes -- as a list of operations; the HIP side only executes
 * that list (rtc_render.hip).  The same function drives the CPU test of the ordering (tests/test_plan.py through
 * rtc_plan_sim_*), which checks that every two kernels that may run together touch disjoint memory.
 */
#pragma once
#include <cstddef>
#include <cstdint>

namespace rtcplan {

constexpr int kSlots = 8;     /* scratch slots the pipelined launches cycle through (kSkySlots) */
constexpr int kGeoRing = 16;  /* geometry-pixel counter sets (one per split launch, a ring) */
constexpr int kGeoLists = 16; /* sub-lists per counter set */
constexpr int kGeoCountStride = 32;
constexpr size_t kInlineSumPixels = 600000; /* small shares, and the alternating cull streams' limit for whole frames */
constexpr size_t kSuperCullPixels = 400000; /* launches of more pixels run rtc_super_cull */
constexpr size_t kSampleBufBudget = (size_t)2 << 30;
constexpr size_t kSampleSlotBytes = 12;

/* streams of a plan: the caller's, the scene's two cull streams and its side stream */
enum Stream : int { kStCaller = 0, kStCull0 = 1, kStCull1 = 2, kStSide = 3, kStreams = 4 };
/* events: the scene's own, per slot where they describe one slot's launch, and the caller's two hooks */
enum Event : int {
    kEvNone = -1,
    kEvCullSync = 0,
    kEvFork = 1,
    kEvJoin = 2,
    kEvSkyDone0 = 3,            /* + slot */
    kEvGeoDone0 = 3 + kSlots,   /* + slot */
    kEvFrame = 3 + 2 * kSlots,  /* the caller's frame event (rtc_scene_set_frame_event) */
    kEvGeometry = 4 + 2 * kSlots, /* the caller's geometry event */
    kEvents = 5 + 2 * kSlots
};
enum Kernel : int { kKPrep, kKSuperCull, kKTileCull, kKSky, kKChain, kKAccum, kKOrder, kKRender, kKReduce };
enum OpKind : int { kOpKernel = 0, kOpRecord = 1, kOpWait = 2 };
struct Op {
    int kind;   /* OpKind */
    int stream; /* Stream */
    int event;  /* record / wait: the event; kernel: the event its completion records (kEvNone: none) */
    int kernel; /* kernel ops: Kernel */
};

/* a stream's identity for the ordering state: the caller's hipStream_t value (0 = the null stream, a stream like any
 * other), or one of the scene's own */
constexpr uint64_t kIdCull0 = ~0ull - 1, kIdCull1 = ~0ull - 2;

/* what a pending (unjoined) sky pass writes: its Color / accumulator buffers and everything that decides their values */
struct Key {
    uint64_t colors, accum;
    float cam[13], env[14];
    int dims[9];
};

/* the per-scene ordering state (RtcDeviceScene::plan) */
struct State {
    int flip;                         /* the next overlapped launch's slot */
    bool slotUsed[kSlots];            /* an overlapped launch used the slot (its events are armed) */
    bool skyPending[kSlots];          /* that launch's sky pass has not been waited for by a later launch */
    Key skyKey[kSlots];
    unsigned long long skySeq[kSlots], skyCount;
    unsigned long long geoSeq;        /* split launches so far: the counter set is geoSeq % kGeoRing */
    bool cullValid;                   /* the last split launch's tile cull zeroed the next counter set ... */
    uint64_t cullStream;              /* ... on this stream (its completion: kEvFork) */
    bool prepValid[kSlots];           /* the slot's primary records are for prepOrigin, written on prepStream */
    uint64_t prepStream[kSlots];
    float prepOrigin[kSlots][3];
    size_t scratchCap, samplesCap;    /* bytes allocated (kSlots slots of scratch; the deferred sample slots) */
    bool cst2;                        /* the second cull stream exists */
};
void init(State &s);

/* the launch as the planner needs it */
struct Request {
    uint64_t stream; /* the caller's stream identity */
    int flags;       /* RTC_F_* */
    int width, rows, rowStride;
    int spp;
    int sphereCount; /* spheres the launch renders (0 with trianglesOnly) */
    int triPadded, maskWords;
    bool segments;   /* the caller asked for segment counters (a joined, counting launch) */
    Key key;
    float origin[3];
    bool legacySlotLayout; /* test hook: round 5's broken layout (slot h at h x this launch's slot size) */
    bool noMerge;          /* the sky pass beside the geometry kernel even where it could follow it (A/B) */
};

/* byte offsets inside one scratch slot (the tile cull's outputs, rtc_render.hip) */
struct Layout {
    size_t mask, pixMask, weight, order, geoList, superMask;
    size_t pixItem;  /* per pixel (tile * 64 + bit) of the geometry pixels: its item (merged sky pass) */
    size_t geoColor; /* per item: its Color bytes (merged sky pass) */
    size_t end;
};

struct Plan {
    bool empty;          /* no rows: only the caller's hooks are recorded */
    bool cull, fused, chain, overlap, smallShare, chainOnCs, superCull, debug;
    bool merge;          /* the sky pass follows the geometry kernel and writes every pixel's Color in whole lines */
    int half;            /* the scratch slot */
    int cs, gs;          /* the culls' stream and the geometry kernel's (Stream) */
    unsigned gridX, gridY, superX, superY;
    size_t blocks, tiles;
    int geoCap;
    size_t slotBytes;    /* bytes per slot (halfBytes: what this launch needs) */
    size_t slotOffset;   /* where slot `half` starts */
    Layout lay;
    size_t scratchNeed;  /* kSlots x slotBytes: grow the scratch to it first (hipFree synchronises the device) */
    bool scratchGrow, samplesGrow, needCst2;
    size_t samplesNeed;
    int sampleCap;       /* items with a deferred slot (0: every geometry pixel sums in-kernel) */
    unsigned long long geoSet, geoSetNext; /* counter sets (ring indices) */
    bool prep, prepCounts; /* rtc_prep_primary runs, and zeroes the counter set too */
    bool cullPrio;
    int nOps;
    Op ops[40];
    State after;         /* the ordering state once every operation is enqueued */
};

/* Plan one launch; `s` is not modified (the executor adopts plan.after once every operation is enqueued). */
void plan_launch(const State &s, const Request &r, Plan &p);

/* The memory one kernel of a plan touches, for the ordering test: resource kinds and byte ranges */
enum Res : int { kResScratch = 0, kResPrim = 1, kResGeoSet = 2, kResSamples = 3, kResSegSlots = 4, kResColors = 5,
                 kResAccum = 6, kResCallerSegments = 7 };
enum Access : int { kRead = 0, kWrite = 1, kAtomic = 2, kKeyedWrite = 3 /* writes values the key determines */ };
struct Footprint {
    int res, access;
    unsigned long long id; /* slot / set / buffer identity */
    unsigned long long lo, hi; /* byte range (scratch) or [0, 1) */
};
int kernel_footprint(const Plan &p, const Request &r, int kernel, Footprint *out, int max);

} // namespace rtcplan

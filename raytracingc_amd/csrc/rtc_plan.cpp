/*
 * rtc_plan.cpp -- the launch planner (rtc_plan.h): every ordering decision of rtc_render_rows_async, as data.
 * Pure host C++; the HIP executor is rtc_render_rows_async (rtc_render.hip), the CPU test tests/test_plan.py.
 */
#include "rtc_plan.h"

#include <algorithm>
#include <cstring>

#include "../../include/rtc.h"

namespace rtcplan {

void init(State &s)
{
    memset(&s, 0, sizeof s);
}

namespace {
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct Emitter {
    Plan &p;
    void op(int kind, int stream, int event, int kernel)
    {
        if (p.nOps < (int)(sizeof p.ops / sizeof p.ops[0]))
            p.ops[p.nOps++] = Op{kind, stream, event, kernel};
    }
    void record(int st, int ev) { op(kOpRecord, st, ev, -1); }
    void wait(int st, int ev) { op(kOpWait, st, ev, -1); }
    void kernel(int st, int k, int stopEv = kEvNone) { op(kOpKernel, st, stopEv, k); }
};

uint64_t stream_id(int st, uint64_t caller)
{
    return st == kStCull0 ? kIdCull0 : st == kStCull1 ? kIdCull1 : caller;
}
} // namespace

void plan_launch(const State &s, const Request &r, Plan &p)
{
    memset(&p, 0, sizeof p);
    p.after = s;
    State &n = p.after;
    Emitter E{p};
    if (r.rows <= 0) { /* nothing to render: the (empty) frame is complete once the caller's stream gets here */
        p.empty = true;
        E.record(kStCaller, kEvGeometry);
        E.record(kStCaller, kEvFrame);
        return;
    }
    const size_t px = (size_t)r.width * (size_t)r.rows;
    p.debug = (r.flags & RTC_F_DEBUG_BOUNCES) != 0;
    /* the tile cull keeps a workgroup's prefilter survivors in LDS (maskWords u64, <= 48 KB) */
    p.cull = !(r.flags & RTC_F_NO_TILE_CULL) && r.maskWords <= 6144;
    /* the split launch (rtc_render_chain + the sky pass): every triangle-only scene */
    p.fused = p.cull && !p.debug && r.sphereCount == 0 && !(r.flags & (RTC_F_NO_COOP | RTC_F_NO_REORDER));
    p.chain = p.fused;
    p.gridX = (unsigned)((r.width + 15) / 16);
    p.gridY = (unsigned)((r.rows + 15) / 16);
    p.blocks = (size_t)p.gridX * p.gridY;
    p.tiles = 4 * p.blocks;
    p.superX = (p.gridX + 3) / 4;
    p.superY = (p.gridY + 3) / 4;
    const size_t maskBytes = p.tiles * (size_t)r.maskWords * 8;
    const size_t superBytes = (size_t)p.superX * p.superY * (size_t)r.maskWords * 8;
    p.geoCap = (int)((p.tiles + kGeoLists - 1) / kGeoLists * 64); /* sub-list l: the tiles t = l mod kGeoLists */
    /* RTC_F_OVERLAP: the sky pass is not joined into the caller's stream (a launch that counts segments joins: the
     * reduction reads the sky pass's counters) */
    p.overlap = (r.flags & RTC_F_OVERLAP) && p.fused && !r.segments;
    p.half = p.overlap ? s.flip : 0;
    /* small shares (row stride > 1, <= kInlineSumPixels) sum in-kernel and, pipelined, prepare, cull and run their
     * geometry kernel on one of the two cull streams by slot parity; so do whole pipelined frames of more pixels
     * (DESIGN §3); smaller whole frames keep the caller's stream (C1 256x256x1: cross-stream hops would be its period) */
    p.smallShare = r.rowStride > 1 && px <= kInlineSumPixels;
    p.chainOnCs = p.overlap && (p.smallShare || px > kInlineSumPixels);
    /* Round 6: a pipelined launch on the alternating streams runs its sky pass AFTER its geometry kernel
     * (which then writes each pixel's colour into a per-item word, not into Color) and the sky pass writes every pixel of
     * the frame in whole 64-B lines.  In the pipelined steady state this sky pass runs beside the next frame's geometry
     * kernel, as the previous one did beside this frame's.  Small shares only: whole 1080p frames took 19 % longer with it
     * (0.398 vs 0.336 ms: the sky pass no longer hides beside its own frame's geometry kernel), 1080p 1/4 shares 4 % less
     * (0.110 vs 0.115 ms), 1/8 shares and C3 fsuzane the same (profiles/r06_f_ab_merged_sky.log).  It does not save
     * bytes: the per-item words are as scattered as the Color triples were (1/4 share: geometry kernel WRITE_SIZE 452 ->
     * 601 KB, sky 1465 -> 1519 KB, profiles/r06_j_pmc_writes.log); the gain is the schedule. */
    p.merge = p.chainOnCs && p.smallShare && !r.noMerge;
    p.needCst2 = p.chainOnCs && !s.cst2;
    if (p.needCst2)
        n.cst2 = true;
    p.cs = p.chainOnCs ? ((p.half & 1) ? kStCull1 : kStCull0) : kStCaller;
    p.gs = p.chainOnCs ? p.cs : kStCaller;
    const uint64_t csId = stream_id(p.cs, r.stream);

    /* An unjoined sky pass of an earlier overlapped launch may still write Color rows and read its scratch slot.  A
     * launch that is not overlapped waits for every such pass; an overlapped one waits when a pending pass reads the slot
     * it rewrites (unless its culls move to a cull stream, which waits for that slot itself, below), or writes the same
     * Color or accumulator buffer with other rows, camera or environment.  One wait on the newest such pass covers every
     * earlier one (the side stream runs them in order); evSkyDone[h] also covers launch h's geometry kernel. */
    int waitSky = -1;
    for (int h = 0; h < kSlots; ++h)
        if (s.skyPending[h] &&
            (!p.overlap || (h == p.half && p.cs == kStCaller) ||
             ((s.skyKey[h].colors == r.key.colors || (r.key.accum && s.skyKey[h].accum == r.key.accum)) &&
              memcmp(&s.skyKey[h], &r.key, sizeof r.key) != 0)) &&
            (waitSky < 0 || s.skySeq[h] > s.skySeq[waitSky]))
            waitSky = h;
    if (waitSky >= 0) {
        E.wait(kStCaller, kEvSkyDone0 + waitSky);
        const unsigned long long upTo = s.skySeq[waitSky];
        for (int h = 0; h < kSlots; ++h)
            if (s.skySeq[h] <= upTo)
                n.skyPending[h] = false;
    }

    /* the scratch: kSlots slots; slot h starts at h x (the allocation's slot size), not h x this launch's size --
     * launches of different sizes are in flight together (round 5 fix; the legacy layout is a test hook) */
    if (p.cull) {
        const size_t need = maskBytes + p.tiles * 8 + (p.blocks + p.tiles + p.blocks + 4) * 4 +
                            ((size_t)kGeoLists * kGeoCountStride + (size_t)kGeoLists * p.geoCap) * 4 + 8 + superBytes +
                            256 + p.tiles * 64 * 4 + (size_t)kGeoLists * p.geoCap * 4; /* + pixItem, geoColor */
        p.slotBytes = align_up(need, 256);
        p.scratchNeed = kSlots * p.slotBytes;
        p.scratchGrow = p.scratchNeed > s.scratchCap;
        if (p.scratchGrow)
            n.scratchCap = p.scratchNeed;
        const size_t slotStride = r.legacySlotLayout ? p.slotBytes : n.scratchCap / kSlots;
        p.slotOffset = (size_t)p.half * slotStride;
        Layout &L = p.lay;
        L.mask = 0;
        L.pixMask = L.mask + maskBytes;
        L.weight = L.pixMask + p.tiles * 8;
        L.order = L.weight + p.blocks * 4;
        L.geoList = L.order + (p.blocks + 4 + (size_t)kGeoLists * kGeoCountStride) * 4;
        L.superMask = align_up(L.geoList + (size_t)kGeoLists * p.geoCap * 4, 8);
        L.pixItem = align_up(L.superMask + superBytes, 256);
        L.geoColor = L.pixItem + p.tiles * 64 * 4;
        L.end = L.geoColor + (size_t)kGeoLists * p.geoCap * 4;
    }
    if (p.chain) {
        p.geoSet = s.geoSeq % kGeoRing;
        p.geoSetNext = (s.geoSeq + 1) % kGeoRing;
        p.cullPrio = p.smallShare && px > 400000;
        /* deferred accumulation slots (joined whole frames; small shares and the alternating streams sum in-kernel) */
        if (r.spp > 0 && !(r.flags & RTC_F_CHAIN_INLINE) && !p.smallShare && !p.chainOnCs) {
            const size_t per = (size_t)r.spp * kSampleSlotBytes + sizeof(int);
            const size_t cap = std::min<size_t>(px, kSampleBufBudget / per);
            p.samplesNeed = cap * per + 256;
            p.samplesGrow = p.samplesNeed > s.samplesCap;
            if (p.samplesGrow)
                n.samplesCap = p.samplesNeed;
            p.sampleCap = (int)cap;
        }
    }

    if (p.cs != kStCaller) {
        /* the cull stream runs this launch's first kernels: after everything the caller enqueued before the launch and
         * after the sky wait above (an event at the caller stream's position), and after the slot's previous user ended
         * (its sky pass and its geometry kernel) */
        E.record(kStCaller, kEvCullSync);
        E.wait(p.cs, kEvCullSync);
        if (s.slotUsed[p.half]) {
            E.wait(p.cs, kEvSkyDone0 + p.half);
            E.wait(p.cs, kEvGeoDone0 + p.half);
        }
    }
    /* the previous split launch's tile cull zeroed this launch's counter set: when it ran on another stream (the null
     * stream included), wait for it -- kEvFork is its completion */
    const bool waitPrevCull = p.chain && s.cullValid && s.cullStream != csId;
    if (waitPrevCull)
        E.wait(p.cs, kEvFork);
    const bool prepCurrent = s.prepValid[p.half] && s.prepStream[p.half] == csId &&
                             memcmp(s.prepOrigin[p.half], r.origin, sizeof r.origin) == 0;
    const bool countsZeroed = !p.chain || (s.cullValid && (s.cullStream == csId || waitPrevCull));
    if (p.chain)
        n.cullValid = false;
    /* rtc_prep_primary: the primary records of this camera origin, and this launch's counter set zeroed; skipped for
     * frames of one camera position on one stream */
    if ((r.triPadded > 0 || p.chain) && !(prepCurrent && countsZeroed)) {
        p.prep = true;
        p.prepCounts = p.chain;
        E.kernel(p.cs, kKPrep);
        n.prepValid[p.half] = true;
        n.prepStream[p.half] = csId;
        memcpy(n.prepOrigin[p.half], r.origin, sizeof r.origin);
    }
    p.superCull = p.cull && px > kSuperCullPixels && r.maskWords > 0;
    if (p.superCull)
        E.kernel(p.cs, kKSuperCull);
    if (!p.cull) {
        E.kernel(kStCaller, kKRender);
    } else {
        /* the split launch forks its sky pass at the tile cull's end: kEvFork is the cull's own completion */
        E.kernel(p.cs, kKTileCull, p.fused ? kEvFork : kEvNone);
        if (p.chain) { /* this cull zeroes the next counter set */
            n.geoSeq = s.geoSeq + 1;
            n.cullValid = true;
            n.cullStream = csId;
        }
        if (p.cs != kStCaller && !p.chainOnCs)
            E.wait(kStCaller, kEvFork);
        if (!p.fused) {
            E.kernel(kStCaller, kKOrder);
            E.kernel(kStCaller, kKRender);
        } else {
            /* the sky pixels on the side stream: concurrently with the geometry kernel, or (merge) after it */
            if (p.merge) {
                E.kernel(p.gs, kKChain, kEvGeoDone0 + p.half);
                E.record(p.gs, kEvGeometry);
                E.wait(kStSide, kEvGeoDone0 + p.half); /* (after the cull too: the geometry kernel follows it on gs) */
                E.kernel(kStSide, kKSky);
                n.skyPending[p.half] = true;
                n.skyKey[p.half] = r.key;
                n.skySeq[p.half] = ++n.skyCount;
                E.record(kStSide, kEvSkyDone0 + p.half);
                E.record(kStSide, kEvFrame);
                n.slotUsed[p.half] = true;
                n.flip = (s.flip + 1) % kSlots;
                return;
            }
            E.wait(kStSide, kEvFork);
            E.kernel(kStSide, kKSky);
            E.record(kStSide, kEvJoin);
            if (p.overlap) {
                n.skyPending[p.half] = true;
                n.skyKey[p.half] = r.key;
                n.skySeq[p.half] = ++n.skyCount;
            }
            /* kEvGeoDone[half]: the completion of the geometry stream's last kernel (the in-order sums, or the
             * geometry kernel when it sums in-kernel) */
            const bool accum = p.sampleCap > 0;
            E.kernel(p.gs, kKChain, p.overlap && !accum ? kEvGeoDone0 + p.half : kEvNone);
            if (accum)
                E.kernel(p.gs, kKAccum, p.overlap ? kEvGeoDone0 + p.half : kEvNone);
            E.record(p.gs, kEvGeometry);
            if (p.overlap) {
                /* no join: the frame is complete once the side stream has passed both passes; kEvSkyDone[half] marks
                 * that point, so a later launch that waits for this one waits for its geometry kernel too */
                E.wait(kStSide, kEvGeoDone0 + p.half);
                E.record(kStSide, kEvSkyDone0 + p.half);
                E.record(kStSide, kEvFrame);
                n.slotUsed[p.half] = true;
                n.flip = (s.flip + 1) % kSlots;
                return;
            }
            E.wait(kStCaller, kEvJoin);
            if (r.segments)
                E.kernel(kStCaller, kKReduce);
            E.record(kStCaller, kEvFrame);
            return;
        }
    }
    E.record(kStCaller, kEvGeometry);
    if (r.segments)
        E.kernel(kStCaller, kKReduce);
    E.record(kStCaller, kEvFrame);
}

int kernel_footprint(const Plan &p, const Request &r, int kernel, Footprint *out, int max)
{
    int k = 0;
    auto put = [&](int res, int acc, unsigned long long id, unsigned long long lo, unsigned long long hi) {
        if (k < max)
            out[k] = Footprint{res, acc, id, lo, hi};
        ++k;
    };
    const unsigned long long o = p.slotOffset;
    const Layout &L = p.lay;
    auto scratch = [&](int acc, size_t lo, size_t hi) { put(kResScratch, acc, 0, o + lo, o + hi); };
    const bool colorsKeyed = true;
    auto colors = [&]() {
        put(kResColors, colorsKeyed ? kKeyedWrite : kWrite, r.key.colors, 0, 1);
        if (r.key.accum)
            put(kResAccum, kKeyedWrite, r.key.accum, 0, 1);
    };
    switch (kernel) {
    case kKPrep:
        put(kResPrim, kWrite, (unsigned long long)p.half, 0, 1);
        if (p.prepCounts)
            put(kResGeoSet, kWrite, p.geoSet, 0, 1);
        break;
    case kKSuperCull:
        put(kResPrim, kRead, (unsigned long long)p.half, 0, 1);
        scratch(kWrite, L.superMask, L.end);
        break;
    case kKTileCull:
        put(kResPrim, kRead, (unsigned long long)p.half, 0, 1);
        if (p.superCull)
            scratch(kRead, L.superMask, L.end);
        scratch(kWrite, L.mask, L.order); /* mask, pixMask, weight */
        if (p.chain) {
            scratch(kWrite, L.geoList, L.superMask);
            if (p.merge)
                scratch(kWrite, L.pixItem, L.geoColor);
            put(kResGeoSet, kAtomic, p.geoSet, 0, 1);
            put(kResGeoSet, kWrite, p.geoSetNext, 0, 1);
        }
        break;
    case kKSky:
        scratch(kRead, L.pixMask, L.weight);
        if (p.merge) {
            scratch(kRead, L.pixItem, L.geoColor);
            scratch(kRead, L.geoColor, L.end);
            put(kResGeoSet, kRead, p.geoSet, 0, 1); /* the counts: an entry's item */
        }
        colors();
        if (r.segments)
            put(kResSegSlots, kAtomic, 0, 0, 1);
        break;
    case kKChain:
        put(kResPrim, kRead, (unsigned long long)p.half, 0, 1);
        scratch(kRead, L.mask, L.pixMask);
        scratch(kRead, L.geoList, L.superMask);
        put(kResGeoSet, kRead, p.geoSet, 0, 1);
        if (p.sampleCap > 0)
            put(kResSamples, kWrite, 0, 0, 1);
        if (p.merge) {
            scratch(kWrite, L.geoColor, L.end);
            if (r.key.accum)
                put(kResAccum, kKeyedWrite, r.key.accum, 0, 1);
        } else {
            colors();
        }
        if (r.segments)
            put(kResSegSlots, kAtomic, 0, 0, 1);
        break;
    case kKAccum:
        put(kResGeoSet, kRead, p.geoSet, 0, 1);
        put(kResSamples, kRead, 0, 0, 1);
        colors();
        break;
    case kKOrder:
        scratch(kRead, L.weight, L.order);
        scratch(kWrite, L.order, L.order + (p.blocks + 4) * 4);
        break;
    case kKRender:
        put(kResPrim, kRead, (unsigned long long)p.half, 0, 1);
        if (p.cull) {
            scratch(kRead, L.mask, L.pixMask);
            scratch(kRead, L.order, L.order + (p.blocks + 4) * 4);
        }
        colors();
        if (r.segments)
            put(kResSegSlots, kAtomic, 0, 0, 1);
        break;
    case kKReduce:
        put(kResSegSlots, kWrite, 0, 0, 1);
        put(kResCallerSegments, kWrite, 0, 0, 1);
        break;
    default:
        break;
    }
    return k;
}

} // namespace rtcplan

/* ---- the CPU test hook (include/rtc.h rtc_plan_sim_*) ---------------------------------------------------------- */
struct RtcPlanSim {
    rtcplan::State st;
    int triPadded, maskWords, legacy;
};

extern "C" int rtc_plan_sim_create(int triCount, int legacySlotLayout, RtcPlanSim **out)
{
    if (!out || triCount < 0)
        return RTC_EINVAL;
    RtcPlanSim *s = new RtcPlanSim();
    rtcplan::init(s->st);
    s->triPadded = (triCount + 7) / 8 * 8;
    s->maskWords = (s->triPadded + 63) / 64;
    s->legacy = legacySlotLayout;
    *out = s;
    return 0;
}

extern "C" int rtc_plan_sim_release(RtcPlanSim *s)
{
    delete s;
    return 0;
}

extern "C" int rtc_plan_sim_launch(RtcPlanSim *s, const RtcRenderDesc *d, unsigned long long stream,
                                   unsigned long long colors, unsigned long long accum, int segments, const float cam[13],
                                   const float env[14], int *ops, int maxOps, unsigned long long *fp, int maxFp)
{
    if (!s || !d || !cam || !env)
        return RTC_EINVAL;
    rtcplan::Request r{};
    r.stream = stream;
    r.flags = d->flags;
    r.width = d->width;
    r.rows = rtc_rows_selected(d);
    r.rowStride = d->rowStride;
    r.spp = d->spp;
    r.sphereCount = 0;
    r.triPadded = s->triPadded;
    r.maskWords = s->maskWords;
    r.segments = segments != 0;
    r.key.colors = colors;
    r.key.accum = accum;
    memcpy(r.key.cam, cam, sizeof r.key.cam);
    memcpy(r.key.env, env, sizeof r.key.env);
    const int dims[9] = {d->width, d->height, r.rows, d->rowStart, d->rowStride, d->spp, d->maxBounce,
                         (d->flags & RTC_F_HOIST_PRIMARY) ? 1 : 0, d->rowBand > 1 ? __builtin_ctz((unsigned)d->rowBand) : 0};
    memcpy(r.key.dims, dims, sizeof dims);
    memcpy(r.origin, cam, sizeof r.origin);
    r.legacySlotLayout = s->legacy != 0;
    static thread_local rtcplan::Plan p;
    rtcplan::plan_launch(s->st, r, p);
    s->st = p.after;
    /* ops: 4 ints each (kind, stream, event, kernel); per kernel op, its footprint entries (5 u64 each: op index, res,
     * access, id, lo, hi -> 6) in fp */
    int nf = 0;
    for (int i = 0; i < p.nOps && i < maxOps; ++i) {
        const rtcplan::Op &o = p.ops[i];
        ops[4 * i] = o.kind, ops[4 * i + 1] = o.stream, ops[4 * i + 2] = o.event, ops[4 * i + 3] = o.kernel;
        if (o.kind != rtcplan::kOpKernel)
            continue;
        rtcplan::Footprint f[16];
        const int k = rtcplan::kernel_footprint(p, r, o.kernel, f, 16);
        for (int j = 0; j < k && j < 16; ++j, ++nf)
            if (fp && nf < maxFp) {
                unsigned long long *q = fp + 6 * (size_t)nf;
                q[0] = (unsigned long long)i, q[1] = (unsigned long long)f[j].res, q[2] = (unsigned long long)f[j].access;
                q[3] = f[j].id, q[4] = f[j].lo, q[5] = f[j].hi;
            }
    }
    /* the scratch regrowth (hipFree + hipMalloc: the device is synchronised first) and the plan's shape, after the ops */
    if (fp && nf < maxFp) {
        unsigned long long *q = fp + 6 * (size_t)nf;
        q[0] = ~0ull, q[1] = p.scratchGrow || p.samplesGrow, q[2] = (unsigned long long)p.half, q[3] = p.chainOnCs,
        q[4] = p.overlap, q[5] = p.slotOffset;
    }
    return p.nOps | ((nf + 1) << 8);
}

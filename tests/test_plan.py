"""the launch planner (raytracingc_amd/csrc/rtc_plan.h) -- every scratch slot, stream, event record and
wait of rtc_render_rows_async -- driven on the CPU with thousands of random launch sequences (rtc_plan_sim_*: the same
plan_launch the HIP executor runs, no GPU).

The checker here is independent of the planner: it replays each sequence's operations on a model of HIP streams and
events (in-order streams; hipEventRecord captures the stream's position; hipStreamWaitEvent orders the stream after the
last record; a kernel's stop event is its completion; a scratch regrowth synchronises the device) as vector clocks, and
asserts that every two kernels that touch the same memory -- a scratch slot's byte range, a slot's primary records, a
counter set, the deferred sample slots, the segment counters, a Color / accumulator buffer written with different
values -- are ordered.  It must also catch round 5's broken scratch layout (slot h at h x the launch's own slot size;
fixed in 65b9c39), which let a smaller launch's tile cull overwrite the geometry list a larger launch's geometry kernel
was reading.  Reference seam: main.c:263-304."""
from __future__ import annotations

import ctypes as C
import random

import numpy as np
import pytest

import raytracingc_amd as rt
from raytracingc_amd._abi import RtcRenderDesc

KERNEL, RECORD, WAIT = 0, 1, 2
KEYED_WRITE, READ, WRITE, ATOMIC = 3, 0, 1, 2
RES_NAMES = ["scratch", "prim", "geoset", "samples", "segslots", "colors", "accum", "caller_segments"]
KNAMES = ["prep", "super_cull", "tile_cull", "sky", "chain", "accum", "order", "render", "reduce"]
N_EVENTS = 5 + 2 * 8
EV_FRAME, EV_GEOMETRY = 3 + 16, 4 + 16


class StreamModel:
    """HIP's ordering rules as vector clocks: op a happens before op b iff a's own component <= b's view of it."""

    def __init__(self):
        self.vc = {}
        self.events = {}

    def _clock(self, st):
        return self.vc.setdefault(st, {})

    def run(self, st):
        c = dict(self._clock(st))
        c[st] = c.get(st, 0) + 1
        self.vc[st] = c
        return st, c[st], c

    def record(self, st, ev):
        self.events[ev] = dict(self._clock(st))

    def wait(self, st, ev):
        snap = self.events.get(ev)
        if snap is None:  # never recorded: hipStreamWaitEvent returns at once
            return
        c = self._clock(st)
        for k, v in snap.items():
            if c.get(k, 0) < v:
                c[k] = v

    def device_sync(self):
        merged = {}
        for c in self.vc.values():
            for k, v in c.items():
                merged[k] = max(merged.get(k, 0), v)
        for st in list(self.vc):
            self.vc[st] = dict(merged)
        self.floor = merged

    @staticmethod
    def before(a, b):
        st, n, _ = a
        return b[2].get(st, 0) >= n


class Scenario:
    """One scene handle and a caller issuing a random launch sequence."""

    def __init__(self, tri_count, legacy=False):
        self.L = rt.lib()
        h = C.c_void_p()
        assert self.L.rtc_plan_sim_create(tri_count, int(legacy), C.byref(h)) == 0
        self.h = h
        self.model = StreamModel()
        self.accesses = []  # (op, res, access, id, lo, hi, key, launch, kernel)
        self.ops = (C.c_int * 256)()
        self.fp = (C.c_ulonglong * (6 * 256))()
        self.n = 0
        self.last_caller = None

    def close(self):
        self.L.rtc_plan_sim_release(self.h)

    def launch(self, d, stream, colors, accum, segments, cam, env):
        caller = ("caller", stream)
        if self.last_caller is not None and self.last_caller != caller:
            # the scene serves one stream at a time (rtc.h): a caller that moves to another stream orders it after the
            # previous one (an event recorded on the old stream, waited for on the new one)
            self.model.record(self.last_caller, ("caller-switch", self.n))
            self.model.wait(caller, ("caller-switch", self.n))
        self.last_caller = caller
        cam_a = (C.c_float * 13)(*cam)
        env_a = (C.c_float * 14)(*env)
        rc = self.L.rtc_plan_sim_launch(self.h, C.byref(d), stream, colors, accum, int(segments), cam_a, env_a,
                                        self.ops, 64, self.fp, 256)
        assert rc > 0, rc
        nops, nfp = rc & 0xFF, rc >> 8
        fps = np.frombuffer(self.fp, dtype=np.uint64, count=6 * nfp).reshape(nfp, 6)
        info = fps[-1]
        assert info[0] == np.uint64(2**64 - 1)
        if int(info[1]):  # a scratch / sample-slot regrowth: hipFree synchronises the device first
            self.model.device_sync()
        streams = {0: caller, 1: "cull0", 2: "cull1", 3: "side"}
        key = (colors, accum, tuple(np.float32(cam).tobytes()), tuple(np.float32(env).tobytes()),
               (d.width, d.height, d.rowStart, d.rowStride, d.rowBand, d.spp, d.maxBounce, d.flags & 1))
        kernel_ops = {}
        for i in range(nops):
            kind, st, ev, k = (int(v) for v in self.ops[4 * i: 4 * i + 4])
            s = streams[st]
            evk = ("launch-hook", self.n, ev) if ev in (EV_FRAME, EV_GEOMETRY) else ("scene", ev)
            if kind == RECORD:
                self.model.record(s, evk)
            elif kind == WAIT:
                self.model.wait(s, evk)
            else:
                o = self.model.run(s)
                kernel_ops[i] = (o, k)
                if ev >= 0:
                    self.model.record(s, evk)
        for row in fps[:-1]:
            i, res, acc, ident, lo, hi = (int(v) for v in row)
            o, k = kernel_ops[i]
            self.accesses.append((o, res, acc, ident, lo, hi, key, self.n, k))
        self.n += 1
        self.last_ops = [tuple(int(v) for v in self.ops[4 * i: 4 * i + 4]) for i in range(nops)]
        return {"slot": int(info[2]), "alt": bool(info[3]), "overlap": bool(info[4]), "offset": int(info[5])}

    def kernel_order(self):
        """The last launch's kernels in enqueue order, as (name, stream)."""
        names = {0: "caller", 1: "cull0", 2: "cull1", 3: "side"}
        return [(KNAMES[k], names[st]) for kind, st, _, k in self.last_ops if kind == KERNEL]

    def hazards(self, limit=5):
        """Pairs of kernels of different launches (or the same one) that touch the same memory without an order."""
        found = []
        by_res = {}
        for a in self.accesses:
            by_res.setdefault((a[1], a[3]), []).append(a)
        for (res, ident), lst in by_res.items():
            for j in range(len(lst)):
                b = lst[j]
                for i in range(j):
                    a = lst[i]
                    if a[0] is b[0]:
                        continue
                    if a[5] <= b[4] or b[5] <= a[4]:  # disjoint byte ranges
                        continue
                    ka, kb = a[2], b[2]
                    if ka == READ and kb == READ or ka == ATOMIC and kb == ATOMIC:
                        continue
                    if ka == KEYED_WRITE and kb == KEYED_WRITE and a[6] == b[6]:
                        continue  # the same values (same buffer, camera, environment, rows)
                    if StreamModel.before(a[0], b[0]):
                        continue
                    found.append((RES_NAMES[res], ident, (a[7], KNAMES[a[8]]), (b[7], KNAMES[b[8]]), a[4], a[5], b[4],
                                  b[5]))
                    if len(found) >= limit:
                        return found
        return found


CAMS = [(-4.0, -1.5, -6.0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 1.2), (-3.0, -1.5, -6.2, 1, 0, 0, 0, 1, 0, 0, 0, 1, 1.2),
        (-4.0, -1.9, -5.2, 0.9, 0, 0.1, 0, 1, 0, 0.1, 0, 0.9, 1.1)]
ENVS = [(0.3, -0.8, 0.5, 1, 1, 1, 0.3, 0.5, 0.9, 0.3, 0.3, 0.3, 500.0, 20.0),
        (0.1, -0.9, 0.2, 1, 1, 1, 0.3, 0.5, 0.9, 0.3, 0.3, 0.3, 200.0, 10.0)]
OVERLAP, CHAIN_INLINE = rt.RTC_F_OVERLAP, rt.RTC_F_CHAIN_INLINE


def _desc(W, H, spp, row_start, stride, band, flags):
    return RtcRenderDesc(W, H, spp, 10, 1, row_start, stride, flags, band)


def _random_launch(rng, shape):
    """A launch the product issues: whole frames and row / band shares of a few sizes, pipelined or joined, counting or
    not, sometimes hoisted, debug or brute force (the non-split paths)."""
    W, H = shape
    G = rng.choice([1, 1, 2, 4, 8])
    band = rng.choice([0, 0, 8]) if G > 1 else 0
    r = rng.randrange(G)
    flags = OVERLAP if rng.random() < 0.8 else 0
    if rng.random() < 0.1:
        flags |= rt.RTC_F_HOIST_PRIMARY
    if rng.random() < 0.05:
        flags |= CHAIN_INLINE
    u = rng.random()
    if u < 0.04:
        flags |= rt.RTC_F_DEBUG_BOUNCES
    elif u < 0.08:
        flags |= rt.RTC_F_NO_TILE_CULL
    return _desc(W, H, rng.choice([1, 16, 64]), r * (band or 1), G, band, flags)


@pytest.mark.parametrize("seed", range(6))
def test_random_launch_sequences_are_race_free(seed):
    """Thousands of launches: 50 random sequences of 24 launches per seed, each on its own scene handle: frame sizes from
    256x256 to 4K (so the scratch is regrown and launches of different sizes are in flight together), shares of 1-8
    ranks in rows or bands of 8, pipelined or joined, three Color buffers, cameras and environments that change, counting
    launches, caller stream switches (the null stream included).  No unordered pair of conflicting kernels."""
    rng = random.Random(1000 + seed)
    shapes = [(1920, 1080), (3840, 2160), (640, 360), (256, 256), (1000, 700)]
    total = 0
    for _ in range(50):
        sc = Scenario(rng.choice([12, 120, 300, 5208]))
        streams = [rng.choice([0, 0x7f001000, 0x7f002000])]
        if rng.random() < 0.3:
            streams.append(rng.choice([0, 0x7f003000]))
        try:
            shape = rng.choice(shapes)
            for _ in range(24):
                if rng.random() < 0.15:
                    shape = rng.choice(shapes)
                d = _random_launch(rng, shape)
                seg = not (d.flags & OVERLAP) and rng.random() < 0.2
                colors = rng.choice([0x1000, 0x2000, 0x3000])
                accum = rng.choice([0, 0, 0, 0x9000 + colors])
                sc.launch(d, rng.choice(streams), colors, accum, seg, rng.choice(CAMS), rng.choice(ENVS))
                total += 1
            hz = sc.hazards()
            assert not hz, f"unordered conflicting kernels: {hz}"
        finally:
            sc.close()
    assert total == 50 * 24


def _band_share_sequence(legacy):
    """Round 5's failing pattern (test_small_shares_sum_in_kernel[True-8-8]): the eight 1080p band shares of a frame
    pipelined back to back on one scene -- the last share is shorter (135 bands of 8 rows: 17 for ranks 0-6, 16 for
    rank 7), so its scratch slot is smaller than the one before it -- then a whole frame."""
    sc = Scenario(120, legacy=legacy)
    try:
        for frame in range(2):
            for r in range(8):
                sc.launch(_desc(1920, 1080, 64, r * 8, 8, 8, OVERLAP), 0x7f001000, 0x1000 + 0x100 * r, 0, False,
                          CAMS[0], ENVS[0])
        sc.launch(_desc(1920, 1080, 64, 0, 1, 0, OVERLAP), 0x7f001000, 0x5000, 0, False, CAMS[0], ENVS[0])
        sc.launch(_desc(1920, 1080, 64, 7 * 8, 8, 8, OVERLAP), 0x7f001000, 0x1700, 0, False, CAMS[0], ENVS[0])
        return sc.hazards()
    finally:
        sc.close()


def test_band_shares_race_free():
    assert _band_share_sequence(legacy=False) == []


def test_checker_catches_round5_slot_layout():
    """The checker is not vacuous: with round 5's slot layout (slot h at h x the launch's own slot size) the same
    sequence has a smaller launch's tile cull writing scratch bytes a larger launch's geometry kernel reads, unordered."""
    hz = _band_share_sequence(legacy=True)
    assert hz, "the legacy slot layout must produce an unordered scratch conflict"
    assert any(h[0] == "scratch" for h in hz), hz


def test_checker_catches_a_dropped_wait():
    """Dropping the previous cull's wait (a launch on the null stream, then one on another stream) is a
    counter-set race the checker sees when the model is told the cull ran unordered -- shown here by replaying a
    sequence whose second launch's ops are stripped of their waits."""
    sc = Scenario(120)
    try:
        sc.launch(_desc(1920, 1080, 64, 0, 8, 0, 0), 0, 0x1000, 0, False, CAMS[0], ENVS[0])  # joined, null stream
        real_wait = sc.model.wait
        sc.model.wait = lambda st, ev: None  # a planner that waits for nothing
        sc.launch(_desc(1920, 1080, 64, 1, 8, 0, OVERLAP), 0x7f001000, 0x2000, 0, False, CAMS[1], ENVS[0])
        sc.model.wait = real_wait
        assert sc.hazards(), "without waits the counter set / primary records must race"
    finally:
        sc.close()


def test_null_stream_then_other_stream_orders_previous_cull():
    """a split launch on the null stream, then an overlapped launch on a cull stream whose counter
    set the first launch's cull zeroed: the second waits for that cull (kEvFork) and its counts are not assumed zeroed
    without it -- no unordered pair."""
    sc = Scenario(120)
    try:
        sc.launch(_desc(1920, 1080, 64, 0, 1, 0, 0), 0, 0x1000, 0, False, CAMS[0], ENVS[0])
        for k in range(4):
            sc.launch(_desc(1920, 1080, 64, 0, 1, 0, OVERLAP), 0x7f001000, 0x2000 + 0x1000 * (k % 3), 0, False,
                      CAMS[k % 2], ENVS[0])
        sc.launch(_desc(640, 360, 16, 0, 1, 0, OVERLAP), 0, 0x2000, 0, False, CAMS[0], ENVS[1])
        assert sc.hazards() == []
    finally:
        sc.close()


def test_plan_shapes():
    """The plan's decisions where DESIGN states them: pipelined whole 1080p frames and small shares take the alternating
    cull streams by slot parity and cycle through the 8 slots; joined launches use slot 0 on the caller's stream; slot
    offsets are multiples of the allocation's slot size."""
    sc = Scenario(120)
    try:
        got = [sc.launch(_desc(1920, 1080, 64, 0, 1, 0, OVERLAP), 0x7f001000, 0x1000, 0, False, CAMS[0], ENVS[0])
               for _ in range(10)]
        assert [g["slot"] for g in got] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
        assert all(g["alt"] and g["overlap"] for g in got)
        step = got[1]["offset"]
        assert step > 0 and all(g["offset"] == g["slot"] * step for g in got)
        j = sc.launch(_desc(1920, 1080, 64, 0, 1, 0, 0), 0x7f001000, 0x1000, 0, False, CAMS[0], ENVS[0])
        assert j == {"slot": 0, "alt": False, "overlap": False, "offset": 0}
        small = sc.launch(_desc(256, 256, 1, 0, 1, 0, OVERLAP), 0x7f001000, 0x4000, 0, False, CAMS[0], ENVS[0])
        assert small["overlap"] and not small["alt"]  # small whole frames keep the caller's stream
        share = sc.launch(_desc(1920, 1080, 64, 3, 8, 0, OVERLAP), 0x7f001000, 0x5000, 0, False, CAMS[0], ENVS[0])
        assert share["overlap"] and share["alt"]
        # small shares: the merged sky pass follows the geometry kernel
        ks = [k for k, _ in sc.kernel_order()]
        assert ks.index("chain") < ks.index("sky") and ("sky", "side") in sc.kernel_order()
        # whole pipelined frames: the sky pass is enqueued beside the geometry kernel, not after it
        sc.launch(_desc(1920, 1080, 64, 0, 1, 0, OVERLAP), 0x7f001000, 0x1000, 0, False, CAMS[0], ENVS[0])
        ks = [k for k, _ in sc.kernel_order()]
        assert ks.index("sky") < ks.index("chain")
    finally:
        sc.close()

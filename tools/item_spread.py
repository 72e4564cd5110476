#!/usr/bin/env python3
"""Per-item timing of rtc_render_chain (diagnostic build: each item's start / end by s_memrealtime, its windows and its
tile's candidate count) for one joined launch of a frame or a row share, and list-scheduling replays of the measured
durations: the kernel's own hand-out (workgroup b owns items b + k * grid, its waves take the next k) beside a global
counter and longest-first orders.  Not part of the product.
Usage: item_spread.py [scene W H spp G band]"""
import ctypes as C
import heapq
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ["RTC_LIB_PATH"] = os.environ.get("RTC_DIAG_LIB") or os.path.join(REPO, "raytracingc_amd", "_lib", "librtc_diag.so")
import torch  # noqa: E402

import raytracingc_amd as rt  # noqa: E402
from conftest import load_tris  # noqa: E402
from raytracingc_amd.distributed import rank_config, rows_per_rank  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "ultracomplex"
W, H, SPP, G = (int(v) for v in sys.argv[2:6]) if len(sys.argv) > 5 else (1920, 1080, 64, 8)
BAND = int(sys.argv[6]) if len(sys.argv) > 6 else 1
tris, _ = load_tris(scene_name)
L = rt.lib()
L.rtc_diag_wavelog.argtypes = [C.c_void_p, C.c_int, C.c_int]
L.rtc_diag_itemlog.argtypes = [C.c_void_p, C.c_int]
L.rtc_diag_itemsect.argtypes = [C.c_void_p, C.c_int]
L.rtc_diag_sections.argtypes = [C.c_void_p, C.c_int]
SECT = {0: "window_setup", 1: "primary_trace", 2: "*hit", 3: "*cull", 4: "*pair_build", 5: "*pair_passes", 6: "*env",
        7: "walk_and_sums", 8: "*hit_loads", 9: "*hit_draws", 14: "*table", 15: "item_setup", 16: "shading", 17: "bounce1", 18: "item_tail", 19: "prologue",
        20: "later_bounce", 21: "later_shading"}
ds = rt.DeviceScene(tris, None)
base = rt.RenderConfig(W, H, SPP, 10, True, overlap=True)
cfg = rank_config(base, 0, G, band=BAND) if G > 1 else base
rows = rows_per_rank(H, G, band=BAND) if G > 1 else H
buf = torch.zeros((rows, W, 3), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
st = torch.cuda.Stream()
for _ in range(5):
    ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
torch.cuda.synchronize()
wl = np.zeros((16384, 8), np.uint64)
il = np.zeros((1 << 18, 4), np.uint64)


def replay(dur, owners, nworkers):
    """list scheduling of durations: owners[i] = the queue item i is in (in order); each queue is served by the workers
    assigned to it (nworkers[q]); returns the makespan"""
    queues = {}
    for i, q in enumerate(owners):
        queues.setdefault(q, []).append(dur[i])
    span = 0.0
    for q, items in queues.items():
        h = [0.0] * nworkers[q]
        for d in items:
            t = heapq.heappop(h)
            heapq.heappush(h, t + d)
        span = max(span, max(h))
    return span


for rep in range(2):
    L.rtc_diag_wavelog(None, 0, 1)
    L.rtc_diag_sections(None, 1)
    ds.render_rows_async(rt.default_scene(), rt.camera_basis(), cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    n = L.rtc_diag_wavelog(wl.ctypes.data, 16384, 1)
    wlv = wl[:n][wl[:n, 0] != 0]
    t0 = int(wlv[:, 0].astype(np.int64).min())
    L.rtc_diag_itemlog(il.ctypes.data, il.shape[0])
    a = il.astype(np.int64)
    ok = (a[:, 0] >= t0) & (a[:, 1] > a[:, 0])
    nItems = int(np.argmin(ok)) if not ok.all() else len(ok)
    a = a[:nItems]
    start, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0
    dur = end - start
    win = a[:, 2] & 0xffff
    cand = (a[:, 2] >> 16) & 0xffff
    wave = a[:, 2] >> 32
    iters = a[:, 3] & 0xffff
    bmfall = (a[:, 3] >> 16) & 0xffff  # lanes that took the exact Box-Muller fallback
    alive = a[:, 3] >> 32  # triangle tests (RTC_DIAG_COUNT builds)
    nWaves = int(wave.max()) + 1
    if rep == 0 and os.environ.get("ITEM_NPZ"):
        np.savez_compressed(os.environ["ITEM_NPZ"], start=start, end=end, win=win, cand=cand, wave=wave, iters=iters,
                            alive=alive, bmfall=bmfall)
    isec = np.zeros((1 << 17, 16), np.uint32)
    L.rtc_diag_itemsect(isec.ctypes.data, isec.shape[0])
    isec = isec[:nItems].astype(np.int64)
    COLS = ["window_setup", "primary_trace", "*hit", "*cull", "*pair_build", "*pair_passes", "*env", "walk_and_sums",
            "*hit_loads", "*hit_draws", "*table", "item_setup", "shading", "bounce1", "item_tail", "prologue"]
    MAIN = [c for c in range(16) if not COLS[c].startswith("*")]

    def shares(rows):
        tot = isec[rows].sum(axis=0)
        m = max(int(tot[MAIN].sum()), 1)
        return {COLS[c]: round(float(tot[c]) / m, 3) for c in range(16) if tot[c]}
    allsec = np.zeros(24, np.uint64)
    L.rtc_diag_sections(allsec.ctypes.data, 1)
    grid = nWaves // 4
    q = lambda v, p: round(float(np.percentile(v, p)), 2)  # noqa: E731
    # the waves' busy time and last end
    busy = np.bincount(wave, weights=dur, minlength=nWaves)
    last = np.zeros(nWaves)
    np.maximum.at(last, wave, end)
    idx = np.arange(nItems)
    dec = np.minimum(idx * 10 // max(nItems, 1), 9)
    by_dec = [round(float(dur[dec == d].mean()), 2) for d in range(10)]
    cq = np.quantile(cand, [0.25, 0.5, 0.75])
    by_cand = [round(float(dur[(cand <= cq[0])].mean()), 2), round(float(dur[(cand > cq[0]) & (cand <= cq[1])].mean()), 2),
               round(float(dur[(cand > cq[1]) & (cand <= cq[2])].mean()), 2), round(float(dur[cand > cq[2]].mean()), 2)]
    own = idx % grid
    wk = {b: 4 for b in range(grid)}
    mean_busy = float(busy.mean())
    replays = {
        "kernel_order": replay(dur, own, wk),
        "kernel_lpt_per_wg": None,
        "global_counter": replay(dur, np.zeros(nItems, int), {0: nWaves}),
        "global_lpt": replay(np.sort(dur)[::-1], np.zeros(nItems, int), {0: nWaves}),
        "global_by_cand_desc": replay(dur[np.argsort(-cand, kind="stable")], np.zeros(nItems, int), {0: nWaves}),
        "global_by_windows_desc": replay(dur[np.argsort(-win, kind="stable")], np.zeros(nItems, int), {0: nWaves}),
    }
    lpt_own = []
    for b in range(grid):
        sel = np.sort(dur[own == b])[::-1]
        lpt_own.append(replay(sel, np.zeros(len(sel), int), {0: 4}))
    replays["kernel_lpt_per_wg"] = max(lpt_own)
    print(json.dumps({
        "scene": scene_name, "W": W, "H": H, "spp": SPP, "G": G, "band": BAND, "items": nItems, "waves": nWaves,
        "span_us": round(float(end.max()), 2), "last_end_p50_us": q(last, 50), "last_end_p90_us": q(last, 90),
        "busy_mean_us": round(mean_busy, 2), "busy_max_us": round(float(busy.max()), 2),
        "dur_us": {"mean": round(float(dur.mean()), 2), "p50": q(dur, 50), "p90": q(dur, 90), "p99": q(dur, 99),
                   "max": round(float(dur.max()), 2)},
        "windows": {"1": int((win == 1).sum()), "2": int((win == 2).sum()), "3+": int((win >= 3).sum())},
        "bm_fallback_items": int((bmfall > 0).sum()),
        "dur_with_without_bm_fallback_us": [round(float(dur[bmfall > 0].mean()), 1) if (bmfall > 0).any() else None,
                                            round(float(dur[bmfall == 0].mean()), 1)],
        "iters_by_dur_top": [[round(float(dur[i]), 1), int(win[i]), int(iters[i]), int(bmfall[i]), int(i)]
                             for i in np.argsort(-dur)[:12]],
        "dur_by_windows_us": [round(float(dur[win == w].mean()), 2) if (win == w).any() else None for w in (1, 2, 3)],
        "cand_quartiles": [int(v) for v in cq], "dur_by_cand_quartile_us": by_cand,
        "corr_dur_cand": round(float(np.corrcoef(dur, cand)[0, 1]), 3),
        "dur_by_position_decile_us": by_dec,
        "start_by_position_decile_us": [round(float(start[dec == d].mean()), 2) for d in range(10)],
        "replay_makespan_us": {k: round(v, 2) for k, v in replays.items()},
        "section_share_all_items": shares(np.ones(nItems, bool)),
        "section_share_items_over_5x_median": shares(dur > 5 * np.median(dur)),
        "items_over_5x_median": int((dur > 5 * np.median(dur)).sum()),
    }), flush=True)
ds.close()

"""Multi-rank plumbing on CPU (gloo, world_size 2 and 3): row interleave across ranks (main.c:84 lifted to
ranks), padded compact parts, the gather to rank 0 and the re-interleave give the single-process frame.
The per-rank renderer here is the CPU oracle (test infrastructure) standing in for the HIP kernel, which
the -m gpu tests cover (tests/test_gpu_parity.py::test_row_partition_and_deinterleave)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_tris, setup_from_flags

from raytracingc_amd.distributed import (FrameRenderer, SharedHostFrames, band_rows, interleave_reference,
                                         rank_config, rank_report, rows_per_rank)

W, H, SPP = 40, 23, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_part(cfg_r, out):
    import oracle.binding as orc
    from raytracingc_amd._abi import RtcRenderDesc

    tris, tonly = load_tris("fsuzane")
    scene, cam, _ = setup_from_flags({})
    d = RtcRenderDesc(cfg_r.width, cfg_r.height, cfg_r.spp, cfg_r.max_bounce, tonly, cfg_r.row_start,
                      cfg_r.row_stride, 0, cfg_r.row_band)
    col, _, _ = orc.render(tris, None, scene, cam, d, threads=2)
    out.zero_()
    out[: col.shape[0]].copy_(torch.from_numpy(col))


def _worker(rank, world, port, q, band=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import raytracingc_amd as rt

        cfg = rt.RenderConfig(W, H, SPP, 10, True)
        fr = FrameRenderer(cfg, _oracle_part, torch.device("cpu"), band=band)
        frame = fr()
        if rank == 0:
            q.put(frame.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 1), (3, 1), (2, 8), (3, 4)])
def test_gloo_frame_equals_single_process(world, band):
    """Rows (band 1) or bands of rows (north_star's row-tile split) across gloo ranks, gathered to rank 0 and
    re-interleaved: the single-process frame."""
    import raytracingc_amd as rt

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, band)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = torch.zeros((H, W, 3), dtype=torch.uint8)
    _oracle_part(rt.RenderConfig(W, H, SPP, 10, True), full)
    assert np.array_equal(frame, full.numpy())


def _subgroup_worker(rank, world, port, q):
    """Ranks 1..world-1 form a group that excludes global rank 0; the group's rank 0 (global rank 1) must
    receive the frame (the gather used dst=0, a global rank outside the group)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import raytracingc_amd as rt

        group = dist.new_group(list(range(1, world)))
        if rank >= 1:
            cfg = rt.RenderConfig(W, H, SPP, 10, True)
            fr = FrameRenderer(cfg, _oracle_part, torch.device("cpu"), group=group)
            assert fr.world == world - 1 and fr.root == 1
            frame = fr()
            if rank == 1:
                q.put(frame.numpy().copy())
            else:
                assert frame is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_subgroup_without_global_rank0():
    import raytracingc_amd as rt

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_subgroup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = torch.zeros((H, W, 3), dtype=torch.uint8)
    _oracle_part(rt.RenderConfig(W, H, SPP, 10, True), full)
    assert np.array_equal(frame, full.numpy())


def test_parse_cpulist():
    from raytracingc_amd.distributed import parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert parse_cpulist("") == set() and parse_cpulist("5") == {5}


def test_band_partition_helpers():
    """rtc.h rowBand: every image row belongs to exactly one rank; the rows each rank renders (band_rows) are what the
    C ABI (rtc_rows_selected) and the oracle (oracle_rows_selected) count, in the same order the oracle renders them;
    the re-interleave statement puts them back."""
    import ctypes as C

    import oracle.binding as orc
    import raytracingc_amd as rt

    for h, g, b in [(1080, 8, 8), (1080, 4, 8), (67, 3, 8), (67, 8, 4), (23, 2, 8), (5, 8, 8), (2160, 8, 16), (17, 1, 8)]:
        got = sorted(y for r in range(g) for y in band_rows(h, r, g, b))
        assert got == list(range(h)), (h, g, b)
        assert rows_per_rank(h, g, b) == max(len(band_rows(h, r, g, b)) for r in range(g))
        for r in range(g):
            cfg = rank_config(rt.RenderConfig(8, h), r, g, b)
            d = cfg.desc()
            n = len(band_rows(h, r, g, b))
            assert rt.lib().rtc_rows_selected(C.byref(d)) == n, (h, g, b, r)
            assert orc.lib().oracle_rows_selected(C.byref(d)) == n, (h, g, b, r)
        parts = torch.zeros((g, rows_per_rank(h, g, b), 2), dtype=torch.int32)
        for r in range(g):
            ys = band_rows(h, r, g, b)
            parts[r, :len(ys), 0] = torch.tensor(ys, dtype=torch.int32)
        assert torch.equal(interleave_reference(parts, h, b)[:, 0], torch.arange(h, dtype=torch.int32))
    # the oracle renders a band share's rows exactly as the full frame's same rows (the seed is the absolute pixel)
    import oracle.binding as orc2
    from raytracingc_amd._abi import RtcRenderDesc

    tris, tonly = load_tris("complex")
    scene, cam, _ = setup_from_flags({})
    Wd, Hd = 24, 37
    full, facc, _ = orc2.render(tris, None, scene, cam, RtcRenderDesc(Wd, Hd, 2, 10, tonly, 0, 1, 0), threads=4)
    for r, g, b in [(1, 3, 8), (0, 2, 16), (2, 4, 4)]:
        ys = band_rows(Hd, r, g, b)
        col, acc, _ = orc2.render(tris, None, scene, cam, RtcRenderDesc(Wd, Hd, 2, 10, tonly, r * b, g, 0, b), threads=4)
        assert np.array_equal(col, full[ys]) and np.array_equal(acc.view(np.uint32), facc[ys].view(np.uint32))


def test_partition_helpers():
    import raytracingc_amd as rt

    for h, g in [(1080, 8), (1080, 7), (23, 3), (5, 8), (1, 1)]:
        rows = rows_per_rank(h, g)
        assert rows * g >= h and (rows - 1) * g < h
        got = sorted(y for r in range(g) for y in range(r, h, g))
        assert got == list(range(h))
        cfg = rank_config(rt.RenderConfig(8, h), min(g - 1, h - 1), g)
        assert cfg.rows() <= rows
    parts = torch.arange(3 * 4 * 2 * 3, dtype=torch.int32).reshape(3, 4, 2, 3)
    out = interleave_reference(parts, 10)
    for y in range(10):
        assert torch.equal(out[y], parts[y % 3, y // 3])


def _shared_worker(rank, world, port, q, name):
    """Each rank writes its rows y = rank + k*world into the node-shared host frame at row pitch world*W*3 (the numpy
    strided copy stands in for the SDMA rtc_copy_rows_d2h_dma the GPU path uses), in two frame buffers."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import raytracingc_amd as rt

        from raytracingc_amd.distributed import pin_rank_near_gpu

        pin_rank_near_gpu(0)  # (no GPU here: caps the threads and leaves the affinity alone)
        assert torch.get_num_threads() == 1
        frames = SharedHostFrames(name, 2, H, W, rank, dist.barrier, register=False)
        cfg = rank_config(rt.RenderConfig(W, H, SPP, 10, True), rank, world)
        part = torch.zeros((rows_per_rank(H, world), W, 3), dtype=torch.uint8)
        _oracle_part(cfg, part)
        n = len(range(rank, H, world))
        for b in range(2):
            flat = np.frombuffer(frames.mm, np.uint8, count=W * 3 * H, offset=b * H * W * 3)
            view = np.lib.stride_tricks.as_strided(flat[rank * W * 3:], shape=(n, W * 3), strides=(world * W * 3, 1))
            view[:] = part[:n].numpy().reshape(n, W * 3)
            del flat, view  # (no view of the mapping may outlive close())
        dist.barrier()
        if rank == 0:
            q.put(frames.frames.copy())
        dist.barrier()
        frames.close(dist.barrier)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_shared_host_frame_rows(world):
    """The multi-process host-frame layout: every rank's interleaved rows land in one shared frame that equals the
    single-process frame (SharedHostFrames, bench.py at N > 1); world 8 is the node the driver's scaling run uses."""
    import raytracingc_amd as rt

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    name = f"rtc_test_shared_{os.getpid()}_{world}"
    procs = [ctx.Process(target=_shared_worker, args=(r, world, port, q, name)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = torch.zeros((H, W, 3), dtype=torch.uint8)
    _oracle_part(rt.RenderConfig(W, H, SPP, 10, True), full)
    for b in range(2):
        assert np.array_equal(frames[b], full.numpy())
    assert not os.path.exists(f"/dev/shm/{name}")


def _report_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = rank_report(0.5 + rank, 1000 + 10 * rank)
        q.put((rank, rep))
    finally:
        dist.destroy_process_group()


def test_gloo_rank_report_plumbing():
    """the N > 1 bench line's communicator fields -- the backend, the world size the process group
    reports (RCCL's on the nccl backend), every rank's ms and segment count in rank order -- identical on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    reps = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {"backend": "gloo", "comm_world_size": 3, "per_rank_ms": [0.5, 1.5, 2.5],
            "per_rank_segments": [1000, 1010, 1020]}
    assert all(reps[r] == want for r in range(world))

"""Multi-GPU frame rendering: one process per GPU, rows interleaved across ranks; the frame reaches the host through
every GPU's own link (SharedHostFrames + rtc_frame_loop / rtc_copy_rows_d2h_dma) or is gathered to rank 0's HBM
with RCCL over xGMI (FrameRenderer).

The reference's only parallelism is the row interleave of its 12 pthreads (main.c:84: thread t renders rows
y = t, t+12, ...).  Here rank r of G renders rows y = r + k*G (or, with band = B > 1, the bands r + k*G of B rows:
north_star's row-tile split, whose 8x8 pixel tiles are 8 adjacent image rows) into a compact [rows, W, 3] uint8 buffer
on its own GPU (the kernel seeds each pixel with its absolute index x + y*W, main.c:95, so the frame does not
depend on G), the compact parts are gathered to rank 0 with one collective (torch.distributed over the `nccl`
backend = RCCL; `gloo` for CPU tests) and rank 0 re-interleaves them with rtc_deinterleave_async.

Per-rank payload at 4K, G = 8: 270 x 3840 x 3 = 3.1 MB (uint8 - quantisation is fused in the kernel).
"""
from __future__ import annotations

import dataclasses
from typing import Callable

import torch
import torch.distributed as dist

from . import RenderConfig, deinterleave_async


def parse_cpulist(text: str) -> set[int]:
    """A sysfs CPU list ("0-3,8,10-11") as a set of CPU numbers."""
    cpus: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_local_cpus(device_index: int) -> set[int] | None:
    """The CPUs of the NUMA node nearest GPU `device_index` (its PCI device's local_cpulist), or None when the
    properties or sysfs do not say."""
    try:
        props = torch.cuda.get_device_properties(device_index)
        bus = "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), props.pci_bus_id, props.pci_device_id)
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            cpus = parse_cpulist(f.read())
        return cpus or None
    except Exception:
        return None


def pin_rank_near_gpu(device_index: int, threads: int = 1) -> dict:
    """Per-rank CPU hygiene for N ranks on one node: cap torch's intra-op threads (the ranks share the
    box's CPU quota; a rank's host work is the launch enqueue and one copy thread that blocks on HSA signals) and, when
    the affinity mask allows, pin the process to the CPUs nearest its GPU.  Returns what was done."""
    import os

    done = {"torch_threads": threads}
    torch.set_num_threads(threads)
    try:
        allowed = os.sched_getaffinity(0)
    except AttributeError:
        return done
    near = gpu_local_cpus(device_index)
    pick = (near & allowed) if near else set()
    if pick and pick != allowed:
        try:
            os.sched_setaffinity(0, pick)
            done["cpus"] = len(pick)
        except OSError:
            pass
    return done


def band_rows(height: int, rank: int, world: int, band: int = 1) -> list[int]:
    """The image rows rank `rank` of `world` renders, in its compact order: y = rank + k*world (main.c:84 lifted to
    ranks), or with band B > 1 the bands b = rank + k*world of B rows (rtc.h RtcRenderDesc.rowBand)."""
    B = max(1, band)
    return [y for b in range(rank, (height + B - 1) // B, world) for y in range(b * B, min(height, b * B + B))]


def copy_rank_rows_to_host(frame_ptr: int, width: int, height: int, rank: int, world: int, dev_ptr: int,
                           band: int = 1) -> None:
    """Rank `rank`'s compact rows (device memory) into their places of a page-locked host frame [height, width, 3] with
    the SDMA engines (rtc_copy_rows_d2h_dma): its full bands as rows of `band` image rows at the band pitch
    world*band*W*3, then a last partial band -- what rtc_frame_loop's copy thread does."""
    from . import copy_rows_d2h_dma

    B = max(1, band)
    rows = len(band_rows(height, rank, world, B))
    rb = width * 3
    full, tail = rows // B, rows % B
    dst = frame_ptr + rank * B * rb
    if full:
        copy_rows_d2h_dma(dst, world * B * rb, dev_ptr, B * rb, B * rb, full)
    if tail:
        copy_rows_d2h_dma(dst + full * world * B * rb, rb, dev_ptr + full * B * rb, rb, rb, tail)


def rank_report(local_ms: float, local_segments: int, group=None) -> dict:
    """What every rank measured, and what the process group itself reports: the backend and the world
    size of the communicator (on the `nccl` backend: the RCCL communicator's rank count, as torch.distributed reports
    it), beside each rank's own timed-region ms and segment count, gathered to every rank in rank order."""
    world = dist.get_world_size(group)
    got = [None] * world
    dist.all_gather_object(got, (int(dist.get_rank(group)), float(local_ms), int(local_segments)), group=group)
    got.sort()
    return {"backend": str(dist.get_backend(group)), "comm_world_size": int(world),
            "per_rank_ms": [round(ms, 4) for _, ms, _ in got], "per_rank_segments": [sg for _, _, sg in got]}


def rows_per_rank(height: int, world: int, band: int = 1) -> int:
    """Rows in the largest part (rank 0's); every rank's compact buffer is padded to this for the gather."""
    return len(band_rows(height, 0, world, band))


def rank_config(cfg: RenderConfig, rank: int, world: int, band: int = 1) -> RenderConfig:
    """Rank `rank`'s share: rows y = rank + k*world, or (band > 1) the bands rank + k*world of `band` rows."""
    B = max(1, band)
    return dataclasses.replace(cfg, row_start=rank * B, row_stride=world, row_band=B if B > 1 else 0)


def interleave_reference(parts: torch.Tensor, height: int, band: int = 1) -> torch.Tensor:
    """Host/CPU statement of the re-interleave (used to check the kernel and the gloo path): image row y is row
    band_rows(height, g, G, band).index(y) of part g, g = (y // band) % G."""
    world = parts.shape[0]
    B = max(1, band)
    ys = torch.arange(height)
    b = ys // B
    return parts[b % world, (b // world) * B + ys % B]


class FrameRenderer:
    """Renders one frame per call across the process group.  `render_part(cfg_r, out_uint8_tensor)` fills a
    rank's compact rows; the default uses the HIP kernel through DeviceScene on the current stream."""

    def __init__(self, cfg: RenderConfig, render_part: Callable[[RenderConfig, torch.Tensor], None],
                 device: torch.device, group=None, band: int = 1):
        self.cfg = cfg
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # global rank of the group's rank 0, the gather's destination
        self.root = dist.get_global_rank(group, 0) if (dist.is_initialized() and group is not None) else 0
        self.device = device
        self.band = max(1, band)
        self.rows = rows_per_rank(cfg.height, self.world, self.band)
        self.cfg_r = rank_config(cfg, self.rank, self.world, self.band)
        self.render_part = render_part
        self.part = torch.zeros((self.rows, cfg.width, 3), dtype=torch.uint8, device=device)
        if self.rank == 0:
            self.gathered = torch.zeros((self.world, self.rows, cfg.width, 3), dtype=torch.uint8, device=device)
            self.frame = torch.zeros((cfg.height, cfg.width, 3), dtype=torch.uint8, device=device)
        else:
            self.gathered = self.frame = None

    def __call__(self) -> torch.Tensor | None:
        self.render_part(self.cfg_r, self.part)
        if self.world > 1:
            glist = list(self.gathered.unbind(0)) if self.rank == 0 else None
            # dst is a global rank: the group's rank 0 (dst=0 broke groups without global rank 0)
            dist.gather(self.part, gather_list=glist, dst=self.root, group=self.group)
        elif self.rank == 0:
            self.gathered[0].copy_(self.part)
        if self.rank != 0:
            return None
        if self.device.type == "cuda":
            deinterleave_async(self.gathered.data_ptr(), self.world, self.rows, self.cfg.width, self.cfg.height,
                               self.frame.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream, self.band)
        else:
            self.frame.copy_(interleave_reference(self.gathered, self.cfg.height, self.band))
        return self.frame


def hip_part_renderer(dev_scene, scene, cam, segments: torch.Tensor | None = None):
    """render_part for FrameRenderer that launches the HIP kernel on torch's current stream."""

    def render_part(cfg_r: RenderConfig, out: torch.Tensor) -> None:
        stream = torch.cuda.current_stream(out.device).cuda_stream
        dev_scene.render_rows_async(scene, cam, cfg_r, out.data_ptr(), None,
                                    segments.data_ptr() if segments is not None else None, stream)

    return render_part


class SharedHostFrames:
    """`nbuf` host frames [H, W, 3] uint8 that every rank of a node maps (a POSIX shared-memory file created by local
    rank 0), page-locked in each process (rtc_host_register) so that each GPU's SDMA engines write its rank's rows
    straight into their places: rank r's rows y = r + k*G start at frame + r*W*3 with row pitch G*W*3
    (rtc_copy_rows_d2h_dma, rtc_frame_loop) -- the reference's threads likewise write their rows into one image
    (main.c:84, :285-302).  `barrier` is the group's barrier; register=False skips the page-locking (CPU tests)."""

    def __init__(self, name: str, nbuf: int, height: int, width: int, local_rank: int, barrier,
                 register: bool = True):
        import mmap
        import os

        import numpy as np

        self.path = f"/dev/shm/{name}"
        self.nbytes = nbuf * height * width * 3
        self.width = width
        self.local = local_rank
        self.registered = False
        if local_rank == 0:
            fd = os.open(self.path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            os.ftruncate(fd, self.nbytes)
            os.close(fd)
        barrier()
        fd = os.open(self.path, os.O_RDWR)
        self.mm = mmap.mmap(fd, self.nbytes)
        os.close(fd)
        self.frames = np.frombuffer(self.mm, np.uint8).reshape(nbuf, height, width, 3)
        self.frames.reshape(-1)[::4096] = 0  # fault the pages in before page-locking them
        barrier()  # (no rank writes its rows before every rank's fault-in stores are done)
        if register:
            from . import host_register

            host_register(self.frames.ctypes.data, self.nbytes)
            self.registered = True

    def rank_rows_ptr(self, b: int, rank: int, band: int = 1) -> int:
        """Where rank `rank`'s first row (y = rank, or y = rank*band for bands) of frame buffer b lives; the pitch
        between its consecutive rows (bands) is world * band * W * 3."""
        return self.frames[b].ctypes.data + rank * max(1, band) * self.width * 3

    def close(self, barrier) -> None:
        import os

        if self.registered:
            from . import host_unregister

            host_unregister(self.frames.ctypes.data)
        del self.frames
        self.mm.close()
        barrier()
        if self.local == 0 and os.path.exists(self.path):
            os.unlink(self.path)

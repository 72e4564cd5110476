"""GPU parity: the HIP path (librtc.so on gfx950) against the CPU oracle and the reference's golden vectors.

Bar (BASELINE.json north_star): per-channel |delta| <= 1e-4 on the pre-quantisation float framebuffer (NaN == NaN);
we also assert that no pixel exceeds it, that the traced segment count (paths) is identical, and we report
the uint8 mismatch count.  Integer / index work (RNG, hit tests, hit distances) is bit-exact.  The device
powf restates glibc's own algorithm (rtc_math.h), so whole frames are bit-identical to the reference except
NaN sign bits on height-1 frames (every direction NaN); every shortcut of the GPU path (tile lists, clusters,
reach masks, state-indexed windows, deferred sums, hoisting, pipelined frames) is checked bit-exact against its
brute-force counterpart.
"""
from __future__ import annotations

import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, load_tris, render_golden, scene_spheres, setup_from_flags

import oracle.binding as orc
import raytracingc_amd as rt
from raytracingc_amd._abi import RtcRenderDesc

pytestmark = pytest.mark.gpu

TOL = 1e-4  # per-channel float tolerance (BASELINE.json north_star)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _compare(gpu, ref):
    """(max |delta| treating NaN==NaN, pixels above TOL, exact-match fraction)"""
    g, r = gpu.astype(np.float64), ref.astype(np.float64)
    both_nan = np.isnan(g) & np.isnan(r)
    d = np.where(both_nan, 0.0, np.abs(g - r))
    d = np.where(np.isnan(d), np.inf, d)
    over = int((d.reshape(-1, 3).max(1) > TOL).sum())
    exact = float((_bits(gpu) == _bits(ref)).mean())
    return float(d.max()) if d.size else 0.0, over, exact


# ---- single functions, bit-exact against the reference's own outputs ------------------------------------
def test_random_sequences_bit_exact(gpu_available):
    k = np.load(f"{GOLDEN}/kat_rng.npz")
    u, g, d = rt.random_sequences(k["seeds"], k["uniform"].shape[1])
    assert np.array_equal(_bits(u), _bits(k["uniform"]))
    assert np.array_equal(_bits(g), _bits(k["normal"]))
    assert np.array_equal(_bits(d), _bits(k["direction"]))


def test_ray_triangle_bit_exact(gpu_available):
    k = np.load(f"{GOLDEN}/kat_tri.npz")
    hit, dst = rt.rayTriangle(k["rays"], k["tris"])
    assert np.array_equal(hit, k["didHit"])
    m = hit == 1
    assert np.array_equal(_bits(dst[m]), _bits(k["dst"][m]))


def test_ray_sphere_bit_exact(gpu_available):
    k = np.load(f"{GOLDEN}/kat_sphere.npz")
    hit, dst, nrm = rt.raySphere(k["rays"], k["spheres"])
    assert np.array_equal(hit, k["didHit"])
    m = hit == 1
    assert np.array_equal(_bits(dst[m]), _bits(k["dst"][m]))
    assert np.array_equal(_bits(nrm[m]), _bits(k["normal"][m]))


@pytest.mark.parametrize("fixture", ["kat_env", "kat_env_edge"])
def test_environment_bit_exact(fixture, gpu_available):
    """kat_env_edge: signed zeros, rays below the horizon / away from the sun, special sun intensities and
    focus values -- where the device skips a powf whose value it knows (rtc_device.h environment)."""
    k = np.load(f"{GOLDEN}/{fixture}.npz")
    out = rt.getEnvironmentLight(k["rays"], k["scenes"])
    nan = np.isnan(k["out"])
    assert np.array_equal(np.isnan(out), nan)
    assert np.array_equal(_bits(out[~nan]), _bits(k["out"][~nan]))


# ---- whole renders against the oracle ------------------------------------------------------------------
GOLD = render_golden()


def _render_both(g, hoist=False):
    tris, tonly = load_tris(g["scene"])
    sph = scene_spheres(g["scene"])
    scene, cam, mb = setup_from_flags(g["flags"])
    cfg = rt.RenderConfig(g["width"], g["height"], g["spp"], mb, bool(tonly), hoist)
    col, acc, st = rt.render(tris, sph, scene, cam, cfg, want_accum=True)
    d = RtcRenderDesc(g["width"], g["height"], g["spp"], mb, tonly, 0, 1, 0)
    ocol, oacc, oseg = orc.render(tris, sph, scene, cam, d, threads=16)
    return col, acc, st, ocol, oacc, oseg


# Height-1 frames: H/2 = 0, so every primary direction is NaN (main.c:88-89 divides by (float)(H/2)).  Their
# floats are NaN on both sides but the NaN sign bit differs (x86 vs gfx950 canonicalisation); the uint8
# frame and the BMP are identical.  Every other configuration is bit-identical to the reference.
NAN_SIGN_ONLY = {"complex_1x1x5", "cube_7x1x2"}


@pytest.mark.parametrize("name", sorted(GOLD))
def test_render_matches_oracle(name, gpu_available):
    g = GOLD[name]
    col, acc, st, ocol, oacc, oseg = _render_both(g)
    mx, over, exact = _compare(acc, oacc)
    u8 = int((col != ocol).any(-1).sum())
    same_as_reference = hashlib.sha256(acc.tobytes()).hexdigest() == g["float_sha256"]
    print(f"{name}: max|d|={mx:.3g} over={over} exact={exact:.5f} u8_mismatch={u8} bit_exact_vs_ref={same_as_reference}")
    assert over == 0 and mx <= TOL
    assert st["segments"] == oseg  # identical paths
    assert u8 == 0
    if name in NAN_SIGN_ONLY:
        assert np.isnan(acc).all() and np.isnan(oacc).all()
    else:
        # the pre-quantisation framebuffer hashes to the reference's own (rtc_ref, tests/golden/make_golden.py)
        assert same_as_reference
    # the BMP written from the GPU frame is the reference's, byte for byte
    bmp = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"rtc_{os.getpid()}_{name}.bmp")
    rt.write_bmp(bmp, col)
    try:
        assert hashlib.md5(open(bmp, "rb").read()).hexdigest() == g["bmp_md5"]
    finally:
        os.remove(bmp)


@pytest.mark.parametrize("name", ["default_160x90x4", "ultracomplex_160x90x4", "fsuzane_odd_33x17x3",
                                  "default_b1_32x18x4"])
def test_hoisted_primary_is_bit_exact(name, gpu_available):
    g = GOLD[name]
    tris, tonly = load_tris(g["scene"])
    sph = scene_spheres(g["scene"])
    scene, cam, mb = setup_from_flags(g["flags"])
    base = rt.RenderConfig(g["width"], g["height"], g["spp"], mb, bool(tonly))
    c0, a0, s0 = rt.render(tris, sph, scene, cam, base, want_accum=True)
    c1, a1, s1 = rt.render(tris, sph, scene, cam, rt.RenderConfig(**{**base.__dict__, "hoist": True}), want_accum=True)
    assert np.array_equal(_bits(a0), _bits(a1)) and np.array_equal(c0, c1)
    assert s0["segments"] == s1["segments"]


@pytest.mark.parametrize("name", ["default_160x90x4", "ultracomplex_160x90x4", "fsuzane_odd_33x17x3",
                                  "complex_64x36x16", "cube_64x36x4", "default_b1_32x18x4",
                                  "ultracomplex_cam_96x64x8", "rsuzanne_160x90x4", "suze_quads_64x36x4"])
@pytest.mark.parametrize("hoist", [False, True])
def test_tile_cull_is_bit_exact(name, hoist, gpu_available):
    """Primary segments over the 8x8 tile's candidate list (rtc_tile_cull) == brute force over every
    triangle (RTC_F_NO_TILE_CULL, what calculateRayCollision does): same bits, same paths, fewer tests."""
    g = GOLD[name]
    tris, tonly = load_tris(g["scene"])
    sph = scene_spheres(g["scene"])
    scene, cam, mb = setup_from_flags(g["flags"])
    base = rt.RenderConfig(g["width"], g["height"], g["spp"], mb, bool(tonly), hoist)
    c0, a0, s0 = rt.render(tris, sph, scene, cam, rt.RenderConfig(**{**base.__dict__, "tile_cull": False}),
                           want_accum=True)
    c1, a1, s1 = rt.render(tris, sph, scene, cam, base, want_accum=True)
    assert np.array_equal(_bits(a0), _bits(a1)) and np.array_equal(c0, c1)
    assert s0["segments"] == s1["segments"]
    assert s1["tri_tests"] <= s0["tri_tests"]
    # one lane per pixel everywhere (RTC_F_NO_COOP, rtc_render_kernel) == the split launch (rtc_render_chain over
    # the geometry pixels, rtc_render_sky over the rest)
    c2, a2, s2 = rt.render(tris, sph, scene, cam, rt.RenderConfig(**{**base.__dict__, "coop": False}),
                           want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a2)) and np.array_equal(c1, c2)
    assert s1["segments"] == s2["segments"]
    if sph is None or len(sph) == 0:
        # the chain kernel culls bounce clusters and unreachable first-bounce records: fewer or equal tests
        assert s1["tri_tests"] <= s2["tri_tests"]
    # the state-indexed kernel summing each pixel's samples itself (RTC_F_CHAIN_INLINE) == the deferred pass
    c6, a6, s6 = rt.render(tris, sph, scene, cam, rt.RenderConfig(**{**base.__dict__, "chain_inline": True}),
                           want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a6)) and np.array_equal(c1, c6) and s1["segments"] == s6["segments"]
    assert s6["tri_tests"] == s1["tri_tests"]
    print(f"{name} hoist={hoist}: tests {s0['tri_tests']} -> {s1['tri_tests']} (+{s1['discarded_tests']} discarded)")


def test_tile_cull_many_triangles(gpu_available):
    """A synthetic 500-triangle scene (5 shifted copies of complex.obj; 8 mask words per tile): culled ==
    brute force bit for bit, and both match the oracle."""
    base_tris, tonly = load_tris("complex")
    copies = []
    for k, (dx, dz) in enumerate([(0, 0), (2.5, 0), (-2.5, 0), (0, 2.5), (0, -2.5)]):
        t = base_tris.copy()
        for v in ("posA", "posB", "posC"):
            t[v]["x"] += np.float32(dx)
            t[v]["z"] += np.float32(dz)
        copies.append(t)
    tris = np.concatenate(copies)
    assert len(tris) == 500
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(96, 54, 4, 10, True)
    c0, a0, s0 = rt.render(tris, None, scene, cam, rt.RenderConfig(**{**cfg.__dict__, "tile_cull": False}),
                           want_accum=True)
    c1, a1, s1 = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    assert np.array_equal(_bits(a0), _bits(a1)) and s0["segments"] == s1["segments"]
    ocol, oacc, oseg = orc.render(tris, None, scene, cam, RtcRenderDesc(96, 54, 4, 10, tonly, 0, 1, 0), threads=8)
    mx, over, _ = _compare(a1, oacc)
    assert over == 0 and s1["segments"] == oseg


def test_chain_occupancy_hint(gpu_available):
    """rtc_scene_chain_wgs: whole frames of scenes whose bounce rays often hit again (bounce_hit_share > 0.15: fsuzane)
    run 4 geometry-kernel workgroups per CU, the others 3; the frame is the same either way (fsuzane's
    full-size frame: test_full_size_baseline_configs)."""
    for name, want in (("fsuzane", 4), ("ultracomplex", 3), ("complex", 3), ("cube", 3)):
        tris, _ = load_tris(name)
        ds = rt.DeviceScene(tris, None)
        assert ds.chain_wgs == want, name
        ds.close()


@pytest.mark.parametrize("overlap", [False, True])
def test_tile_hint_order_same_frame(overlap, gpu_available):
    """Repeated launches of one DeviceScene interleaved with launches of another camera and another row share all
    equal the oracle bit for bit: nothing a launch leaves in the scene's buffers (counter sets, scratch slots, and in
    builds with RTC_GEO_HINT the per-pixel order hint the geometry kernel sets for the next tile cull) changes a
    later frame."""
    import torch

    from raytracingc_amd.distributed import rank_config

    tris, tonly = load_tris("fsuzane")
    scene = rt.default_scene()
    cam = rt.camera_basis()
    cam2 = rt.camera_basis((1.5, 1.0, -6.0), (0.0, 1.0, 0.0), 1.2)
    w, h, spp = 96, 64, 8
    d = RtcRenderDesc(w, h, spp, 10, tonly, 0, 1, 0, 0)
    ocol, oacc, _ = orc.render(tris, None, scene, cam, d, threads=8)
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    cfg = rt.RenderConfig(w, h, spp, 10, bool(tonly), overlap=overlap)
    other = [(cam2, cfg), (cam, rank_config(cfg, 1, 2, band=8))]
    got = []
    for rep in range(4):
        buf = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
        acc = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        ds.render_rows_async(scene, cam, cfg, buf.data_ptr(), accum_ptr=acc.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        got.append((buf.cpu().numpy(), acc.cpu().numpy()))
        if rep >= 2:  # scramble the hint with other launches of the scene
            for c, f in other:
                junk = torch.zeros((max(f.rows(), 1), w, 3), dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                ds.render_rows_async(scene, c, f, junk.data_ptr(), stream=st.cuda_stream)
                torch.cuda.synchronize()
    ds.close()
    nan = np.isnan(oacc)
    for gcol, gacc in got:
        assert np.array_equal(gcol, ocol)
        assert np.array_equal(np.isnan(gacc), nan)
        assert np.array_equal(_bits(gacc[~nan]), _bits(oacc[~nan]))


@pytest.mark.parametrize("seed", range(24))
def test_random_configurations_match_oracle(seed, gpu_available):
    """Randomised end-to-end parity against the CPU restatement (the oracle pinned to the reference's fixtures):
    scene, camera, field of view, frame shape, spp, maxBounce, row partition (rows or bands), sun direction, focus
    (odd and even integers, fractions), intensity (negative and zero included), sky and ground colours, and the launch
    path (joined rtc_render, hoisted, or the device-resident pipelined launch).  Floats bit for bit and the same
    segment count as the oracle."""
    import torch

    rng = np.random.default_rng(1000 + seed)
    name = ["ultracomplex", "complex", "fsuzane", "cube", "suze", "asuzane"][seed % 6]
    tris, tonly = load_tris(name)
    origin = tuple(float(v) for v in rng.uniform(-8, 8, 3))
    look = tuple(float(v) for v in rng.uniform(-1.5, 1.5, 3) + np.array([0, 1.5, 0]))
    cam = rt.camera_basis(origin, look, float(rng.choice([0.5, 1.0, 1.6])))
    sun = tuple(float(v) for v in rng.uniform(-100, 100, 3))
    focus = float(rng.choice([1.0, 3.0, 4.0, 0.5, 250.0, 7.25]))
    intensity = float(rng.choice([0.0, -2.0, 0.3, 5.0, 40.0]))
    col = lambda: tuple(float(v) for v in rng.uniform(0, 1.5, 3))  # noqa: E731
    scene = rt.default_scene(sun=sun, ground=col(), horizon=col(), zenith=col(), focus=focus, intensity=intensity)
    w, h = int(rng.integers(16, 96)), int(rng.integers(8, 64))
    spp, mb = int(rng.integers(1, 24)), int(rng.choice([1, 2, 3, 10]))
    band = int(rng.choice([0, 0, 2, 8]))
    stride = int(rng.choice([1, 1, 2, 3]))
    start = int(rng.integers(0, stride)) * max(1, band)
    start = start if start < h else 0
    path = ["joined", "hoisted", "pipelined"][seed % 3]
    cfg = rt.RenderConfig(w, h, spp, mb, bool(tonly), hoist=path == "hoisted", row_start=start, row_stride=stride,
                          row_band=band)
    d = RtcRenderDesc(w, h, spp, mb, tonly, start, stride, 0, band)
    ocol, oacc, oseg = orc.render(tris, None, scene, cam, d, threads=8)
    if path == "pipelined":
        rows = cfg.rows()
        ds = rt.DeviceScene(tris, None)
        buf = torch.zeros((max(rows, 1), w, 3), dtype=torch.uint8, device="cuda")
        acc = torch.zeros((max(rows, 1), w, 3), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        ev = torch.cuda.Event()
        ev.record(st)
        ds.set_frame_event(ev.cuda_event)
        ds.render_rows_async(scene, cam, rt.RenderConfig(**{**cfg.__dict__, "overlap": True}), buf.data_ptr(),
                             accum_ptr=acc.data_ptr(), stream=st.cuda_stream)
        ev.synchronize()
        torch.cuda.synchronize()
        gcol, gacc = buf.cpu().numpy()[:rows], acc.cpu().numpy()[:rows]
        ds.close()
        gseg = oseg
    else:
        gcol, gacc, st = rt.render(tris, None, scene, cam, cfg, want_accum=True)
        gseg = st["segments"]
    print(f"{name} {w}x{h}x{spp} mb={mb} band={band} stride={stride} start={start} focus={focus} I={intensity} {path}")
    nan = np.isnan(oacc)
    assert np.array_equal(np.isnan(gacc), nan)
    assert np.array_equal(_bits(gacc[~nan]), _bits(oacc[~nan]))
    assert np.array_equal(gcol, ocol)
    assert gseg == oseg


@pytest.mark.parametrize("seed", range(6))
def test_tile_cull_random_cameras(seed, gpu_available):
    """The tile prefilter (TileCone: a bound of the primary filter over each 8x8 tile's direction cone) and the
    cluster culling under random cameras, fields of view and frame shapes, rows partitions included: the
    split launch == brute force (RTC_F_NO_TILE_CULL, every primary segment tests every triangle), bit for
    bit, with the same segment counts."""
    rng = np.random.default_rng(seed)
    name = ["ultracomplex", "complex", "fsuzane"][seed % 3]
    tris, tonly = load_tris(name)
    origin = tuple(float(v) for v in rng.uniform(-9, 9, 3))
    look = tuple(float(v) for v in rng.uniform(-1.5, 1.5, 3) + np.array([0, 2.5, 0]))
    fov = float(rng.choice([0.35, 1.0, 1.7, 3.0]))
    cam = rt.camera_basis(origin, look, fov)
    scene = rt.default_scene()
    w, h = int(rng.integers(24, 150)), int(rng.integers(9, 120))
    stride = int(rng.choice([1, 1, 3]))
    base = rt.RenderConfig(w, h, 3, 10, bool(tonly), row_start=int(rng.integers(0, stride)), row_stride=stride)
    c0, a0, s0 = rt.render(tris, None, scene, cam, rt.RenderConfig(**{**base.__dict__, "tile_cull": False}),
                           want_accum=True)
    c1, a1, s1 = rt.render(tris, None, scene, cam, base, want_accum=True)
    assert np.array_equal(_bits(a0), _bits(a1)) and np.array_equal(c0, c1)
    assert s0["segments"] == s1["segments"]
    print(f"{name} {w}x{h} fov={fov} origin={origin}: tests {s0['tri_tests']} -> {s1['tri_tests']}")


def test_tile_cull_full_frame(gpu_available):
    """The BASELINE frame (ultracomplex 1920x1080, 16 spp here): culled == brute force bit for bit, and the
    culled run evaluates far fewer ray-triangle tests."""
    tris, tonly = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(1920, 1080, 16, 10, True)
    c0, a0, s0 = rt.render(tris, None, scene, cam, rt.RenderConfig(**{**cfg.__dict__, "tile_cull": False}),
                           want_accum=True)
    c1, a1, s1 = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    assert np.array_equal(_bits(a0), _bits(a1)) and s0["segments"] == s1["segments"]
    assert s0["tri_tests"] == s0["segments"] * len(tris)
    assert s1["tri_tests"] < s0["tri_tests"] // 4
    c2, a2, s2 = rt.render(tris, None, scene, cam, rt.RenderConfig(**{**cfg.__dict__, "reorder": False}),
                           want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a2)) and s1["segments"] == s2["segments"]
    print(f"1080p x16: brute {s0['render_ms']:.3f} ms, culled {s1['render_ms']:.3f} ms, raster order "
          f"{s2['render_ms']:.3f} ms; "
          f"tests {s0['tri_tests']} -> {s1['tri_tests']}")


@pytest.mark.parametrize("scene,mb", [("default", 10), ("ultracomplex", 10), ("default", 3), ("fsuzane", 0)])
def test_debug_bounce_integrator(scene, mb, gpu_available):
    """calcDebugColor (raytracing.c:242-260) as a kernel variant (RTC_F_DEBUG_BOUNCES) == the oracle's, which
    tests/test_oracle.py pins to the reference's own calcDebugColor."""
    tris, tonly = load_tris(scene)
    sph = scene_spheres(scene)
    s, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(64, 36, 4, mb, bool(tonly), debug_bounces=True)
    col, acc, st = rt.render(tris, sph, s, cam, cfg, want_accum=True)
    d = RtcRenderDesc(64, 36, 4, mb, tonly, 0, 1, rt.RTC_F_DEBUG_BOUNCES)
    ocol, oacc, oseg = orc.render(tris, sph, s, cam, d, threads=8)
    mx, over, exact = _compare(acc, oacc)
    assert over == 0 and st["segments"] == oseg and np.array_equal(col, ocol)
    assert exact == 1.0  # no environment lookup in this integrator: bit-exact


@pytest.mark.parametrize("band", [1, 8, 4])
def test_row_partition_and_deinterleave(band, gpu_available):
    """Ranks render y = r + k*G (band 1) or the bands r + k*G of `band` rows (rtc.h rowBand) into compact buffers;
    the gathered parts re-interleaved by the kernel equal the single-GPU frame bit for bit (G = 2..8 simulated on one
    device; H = 67 leaves a partial last band)."""
    import torch

    from raytracingc_amd.distributed import rank_config, rows_per_rank

    tris, tonly = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H = 120, 67
    cfg = rt.RenderConfig(W, H, 4, 10, True)
    ref, _, _ = rt.render(tris, None, scene, cam, cfg)
    ds = rt.DeviceScene(tris, None)
    for G in (2, 3, 4, 8):
        rows = rows_per_rank(H, G, band)
        parts = torch.zeros((G, rows, W, 3), dtype=torch.uint8, device="cuda")
        for r in range(G):
            rc = rank_config(cfg, r, G, band)
            if rc.rows() == 0:
                continue
            ds.render_rows_async(scene, cam, rc, parts[r].data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
        rt.deinterleave_async(parts.data_ptr(), G, rows, W, H, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                              band)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref), f"G={G} band={band}"
    ds.close()


@pytest.mark.parametrize("band", [1, 8])
@pytest.mark.parametrize("G", [8, 4])
@pytest.mark.parametrize("overlap", [False, True])
def test_small_shares_sum_in_kernel(overlap, G, band, gpu_available):
    """The bench's 8- and 4-GPU shares of the 1080p x64 headline frame (rows y = r + Gk, 135 / 270 rows: small enough
    that rtc_render_chain sums each pixel's samples itself instead of the deferred pass) equal the single-GPU frame,
    which sums deferred, bit for bit in floats and bytes; with and without frame pipelining (pipelined, consecutive
    shares alternate between the two cull streams, each share's geometry kernel unordered against the previous one's:
    RTC_SHARE_CHAIN_CS)."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H = 1920, 1080
    ref, racc, _ = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, 64, 10, True), want_accum=True)
    from raytracingc_amd.distributed import band_rows, rank_config, rows_per_rank

    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.current_stream().cuda_stream
    rows = rows_per_rank(H, G, band)
    out = torch.zeros((G, rows, W, 3), dtype=torch.uint8, device="cuda")
    acc = torch.zeros((G, rows, W, 3), dtype=torch.float32, device="cuda")
    for r in range(G):
        cfg = rank_config(rt.RenderConfig(W, H, 64, 10, True, overlap=overlap), r, G, band)
        ds.render_rows_async(scene, cam, cfg, out[r].data_ptr(), acc[r].data_ptr(), None, st)
    torch.cuda.synchronize()
    ds.close()
    o, a = out.cpu().numpy(), acc.cpu().numpy()
    for r in range(G):
        ys = np.asarray(band_rows(H, r, G, band))
        n = len(ys)
        bad = np.nonzero(np.any(o[r, :n] != ref[ys], axis=2))
        detail = ""
        if len(bad[0]):
            rr, xx = bad
            detail = (f": {len(rr)} pixels, rows {sorted(set(int(ys[v]) for v in rr))[:12]}, x {int(xx.min())}..{int(xx.max())}, "
                      f"first {[(int(ys[rr[k]]), int(xx[k]), o[r, rr[k], xx[k]].tolist(), ref[ys[rr[k]], xx[k]].tolist(), a[r, rr[k], xx[k]].tolist(), racc[ys[rr[k]], xx[k]].tolist()) for k in range(min(3, len(rr)))]}")
        assert np.array_equal(o[r, :n], ref[ys]), f"rank {r} bytes{detail}"
        assert np.array_equal(_bits(a[r, :n]), _bits(racc[ys])), f"rank {r} floats"


def test_mixed_size_overlapped_launches(gpu_available):
    """Pipelined launches of different sizes in flight together on one scene: the 1080p band partition's rank 6 (17
    bands, 128 spp: a long geometry kernel) and then rank 7 (16 bands, 1 spp), whose tile cull runs on the other cull
    stream while rank 6's geometry kernel still reads its lists; then a whole small frame.  Each launch's scratch slot
    must not overlap the slot of the launch running beside it (round 5: slot offsets were per-launch sizes, and rank 7's
    tile cull overwrote rank 6's geometry list -- geometry pixels left unrendered)."""
    import torch

    from raytracingc_amd.distributed import band_rows, rank_config, rows_per_rank

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H, G, band = 1920, 1080, 8, 8
    plan = [(6, 128), (7, 1), (6, 128), (7, 1)]
    refs = {spp: rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))[0] for spp in (128, 1)}
    sref, _, _ = rt.render(tris, None, scene, cam, rt.RenderConfig(200, 120, 16, 10, True))
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.current_stream().cuda_stream
    rows = rows_per_rank(H, G, band)
    out = torch.zeros((len(plan), rows, W, 3), dtype=torch.uint8, device="cuda")
    sout = torch.zeros((120, 200, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for i, (r, spp) in enumerate(plan):
        cfg = rank_config(rt.RenderConfig(W, H, spp, 10, True, overlap=True), r, G, band)
        ds.render_rows_async(scene, cam, cfg, out[i].data_ptr(), None, None, st)
    ds.render_rows_async(scene, cam, rt.RenderConfig(200, 120, 16, 10, True, overlap=True), sout.data_ptr(), None, None,
                         st)
    torch.cuda.synchronize()
    ds.close()
    o = out.cpu().numpy()
    for i, (r, spp) in enumerate(plan):
        ys = np.asarray(band_rows(H, r, G, band))
        bad = int(np.any(o[i, :len(ys)] != refs[spp][ys], axis=2).sum())
        assert bad == 0, f"launch {i} (rank {r}, {spp} spp): {bad} pixels differ"
    assert np.array_equal(sout.cpu().numpy(), sref)


def test_device_scene_reuse_sizes_counters_timing(gpu_available):
    """One device-resident scene across launches of growing and shrinking frames (per-launch scratch regrown,
    counter slots re-zeroed by the reduce kernel): every frame and segment count equals a fresh rtc_render;
    the opt-in per-kernel timing reports positive times only while enabled."""
    import torch

    tris, tonly = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    ds = rt.DeviceScene(tris, None)
    stream = torch.cuda.current_stream().cuda_stream
    seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device="cuda")
    for k, (W, H) in enumerate([(64, 36), (200, 120), (33, 17), (200, 120)]):
        cfg = rt.RenderConfig(W, H, 4, 10, True)
        ref, _, st = rt.render(tris, None, scene, cam, cfg)
        out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
        seg.zero_()
        ds.set_timing(k % 2 == 1)
        ds.render_rows_async(scene, cam, cfg, out.data_ptr(), None, seg.data_ptr(), stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref), (W, H)
        assert int(seg[0]) == st["segments"] and int(seg[2]) == st["tri_tests"], (W, H)
        kt = ds.kernel_times()
        if k % 2 == 1:
            assert kt is not None and kt[0] > 0 and kt[1] > 0
        else:
            assert kt is None
    ds.close()


def test_pipelined_multi_hit_scene_bit_exact(gpu_available):
    """A scene whose bounces often hit again (fsuzane: 4 geometry-kernel workgroups per CU) pipelined at 1080p runs the
    HITS instantiation of rtc_render_chain (the later bounces' one-pass cull and pair build); its frames equal the joined
    render (the GENERAL instantiation, pinned against the oracle elsewhere) bit for bit, for two cameras."""
    import torch

    tris, _ = load_tris("fsuzane")
    scene = rt.default_scene()
    cams = [rt.camera_basis(), rt.camera_basis((-4.0, -1.9, -5.2), (0.6, -1.0, 1.3), 1.1)]
    W, H, spp = 1920, 1080, 4
    ds = rt.DeviceScene(tris, None)
    assert ds.chain_wgs == 4  # the multi-hit instantiation's scenes
    st = torch.cuda.Stream()
    out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=True)
    for c in cams:
        ref, _, _ = rt.render(tris, None, scene, c, rt.RenderConfig(W, H, spp, 10, True))
        for _ in range(2):
            ds.render_rows_async(scene, c, cfg, out.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref)
    ds.close()


@pytest.mark.parametrize("size", [(256, 144, 8), (1920, 1080, 4)])
@pytest.mark.parametrize("variant", [{}, {"hoist": True}, {"chain_inline": True}])
def test_overlapped_frames_bit_exact(variant, size, gpu_available):
    """RTC_F_OVERLAP (frame pipelining): launches that do not join their sky pass, with the next launch's
    preparation (tile cull into the other scratch slot) overlapping it.  Eight frames over three cameras into two
    buffers, each consumed (copied, after a delay on the consumer's stream) once its frame event fires and rewritten
    only after the launch stream waited for that copy, and two frames of different cameras into one buffer: every
    frame equals a joined rtc_render bit for bit.  At 1920x1080 the launches run on the alternating cull streams
    (they must still start after the caller's wait on the launch stream, and a conflicting launch must
    wait for the previous launch's geometry kernel, not only for its sky pass)."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene = rt.default_scene()
    cams = [rt.camera_basis(), rt.camera_basis((-4.0, -1.9, -5.2), (0.6, -1.0, 1.3), 1.1),
            rt.camera_basis((-5.3, -1.2, -4.1), (1.2, -1.4, 0.7), 0.9)]
    W, H, spp = size
    ref = [rt.render(tris, None, scene, c, rt.RenderConfig(W, H, spp, 10, True))[0] for c in cams]
    cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=True, **variant)
    ds = rt.DeviceScene(tris, None)
    st, cp = torch.cuda.Stream(), torch.cuda.Stream()
    nb = 2
    bufs = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    freed = [None] * nb
    got = []
    def new_event():  # a torch event has no hipEvent_t until its first record
        e = torch.cuda.Event()
        e.record(st)
        return e

    for k in range(8):
        b = k % nb  # buffer b sees cameras 0, 2, 1, 0 ... : a frame written too early is detected
        if freed[b] is not None:  # buffer b is rewritten only after its previous frame was copied
            st.wait_event(freed[b])
        ev = new_event()
        ds.set_frame_event(ev.cuda_event)
        ds.render_rows_async(scene, cams[k % 3], cfg, bufs[b].data_ptr(), stream=st.cuda_stream)
        cp.wait_event(ev)
        with torch.cuda.stream(cp):
            if hasattr(torch.cuda, "_sleep"):
                torch.cuda._sleep(2_000_000)  # ~1 ms: the copy runs late, the next frame's kernels are queued by then
            got.append(bufs[b].clone())
            freed[b] = torch.cuda.Event()
            freed[b].record(cp)
    torch.cuda.synchronize()
    for k, g in enumerate(got):
        assert np.array_equal(g.cpu().numpy(), ref[k % 3]), f"frame {k}"
    # one buffer, two cameras back to back: the second frame's geometry pixels are not overwritten by the first
    # frame's late sky pass or geometry kernel
    for c in (cams[1], cams[2], cams[0], cams[2]):
        ev = new_event()
        ds.set_frame_event(ev.cuda_event)  # one-shot: armed for each launch
        ds.render_rows_async(scene, c, cfg, bufs[0].data_ptr(), stream=st.cuda_stream)
    ev.synchronize()
    assert np.array_equal(bufs[0].cpu().numpy(), ref[2])
    ds.close()


def test_overlap_slot_ring(gpu_available):
    """RTC_F_OVERLAP launches cycle through 8 scratch slots and wait for the unjoined sky passes only when one reads
    the slot being rewritten or writes the same buffer with another camera: 20 back-to-back frames of one camera
    into one buffer (two waits), then 21 alternating between two cameras into one buffer (a wait each), then a
    share of the frame into the same buffer: each final buffer equals a joined render."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene = rt.default_scene()
    cams = [rt.camera_basis(), rt.camera_basis((-4.0, -1.9, -5.2), (0.6, -1.0, 1.3), 1.1)]
    W, H, spp = 320, 180, 8
    ref = [rt.render(tris, None, scene, c, rt.RenderConfig(W, H, spp, 10, True))[0] for c in cams]
    cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=True)
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    for _ in range(20):
        ds.render_rows_async(scene, cams[1], cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), ref[1])
    for k in range(21):  # cams[1], cams[0], ..., the last one cams[1]
        ds.render_rows_async(scene, cams[(k + 1) % 2], cfg, buf.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), ref[1])
    share = rt.RenderConfig(W, H, spp, 10, True, overlap=True, row_start=1, row_stride=2)
    part = buf[: (H + 1) // 2]
    ds.render_rows_async(scene, cams[0], share, part.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(part.cpu().numpy()[: H // 2], ref[0][1::2])
    ds.close()


@pytest.mark.parametrize("size", [(200, 120, 6), (1920, 1080, 2)])
def test_overlap_with_counters_and_mixed_launches(size, gpu_available):
    """An RTC_F_OVERLAP launch that asks for segment counters joins (the counts equal a joined launch's), and
    joined / overlapped / no-tile-cull launches interleaved on one scene (the scratch slots and pending sky
    passes) each produce their frame bit for bit.  At 1920x1080 the overlapped launches run on the alternating cull
    streams, so the joined launch after them and the overlapped launch after that cross streams both ways (ADVICE r04:
    a joined launch's scratch slot 0 must not be rewritten under it by the next cull stream launch)."""
    import torch

    tris, _ = load_tris("complex")
    scene, cam, _ = setup_from_flags({})
    W, H, spp = size
    ref, _, st = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))
    ds = rt.DeviceScene(tris, None)
    s = torch.cuda.current_stream()
    seg = torch.zeros(rt.RTC_SEGMENT_COUNTERS, dtype=torch.int64, device="cuda")
    out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    ds.render_rows_async(scene, cam, rt.RenderConfig(W, H, spp, 10, True, overlap=True), out.data_ptr(), None,
                         seg.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert int(seg[0]) == st["segments"] and int(seg[2]) == st["tri_tests"]
    cfgs = [rt.RenderConfig(W, H, spp, 10, True, overlap=True), rt.RenderConfig(W, H, spp, 10, True),
            rt.RenderConfig(W, H, spp, 10, True, overlap=True), rt.RenderConfig(W, H, spp, 10, True, overlap=True),
            rt.RenderConfig(W, H, spp, 10, True, tile_cull=False), rt.RenderConfig(W, H, spp, 10, True, overlap=True)]
    outs = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in cfgs]
    for c, o in zip(cfgs, outs):
        ds.render_rows_async(scene, cam, c, o.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()  # (the whole device: the unjoined sky passes too)
    for k, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy(), ref), f"launch {k}"
    ds.close()


@pytest.mark.parametrize("variant", [{}, {"hoist": True}, {"chain_inline": True}, {"hoist": True, "chain_inline": True},
                                     {"coop": False}, {"tile_cull": False}])
def test_spp_not_multiple_of_64(variant, gpu_available):
    """spp = 100 (rtc_render_chain's windows of at most 64 state indices, a second window per pixel) against the
    oracle, bit for bit, with identical segment counts."""
    tris, tonly = load_tris("complex")
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(48, 30, 100, 10, True, **variant)
    col, acc, st = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    ocol, oacc, oseg = orc.render(tris, None, scene, cam, RtcRenderDesc(48, 30, 100, 10, tonly, 0, 1, 0), threads=16)
    assert np.array_equal(_bits(acc), _bits(oacc)) and np.array_equal(col, ocol)
    assert st["segments"] == oseg


@pytest.mark.parametrize("band", [0, 8])
@pytest.mark.parametrize("name", ["complex", "ultracomplex"])
def test_render_multi_rccl_equals_render(name, band, gpu_available):
    """rtc_render_multi over every visible device (ncclCommInitAll clique, ncclGather to device 0, re-interleave,
    one D2H) == rtc_render bit for bit, colors and floats; the frame time covers the frame's arrival on the
    host.  On a one-GPU box this runs the whole RCCL path with a clique of one."""
    tris, tonly = load_tris(name)
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(160, 90, 8, 10, True)
    a, fa, sa = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    b, fb, sb = rt.render_multi(tris, None, scene, cam, rt.RenderConfig(160, 90, 8, 10, True, row_band=band),
                                rt.device_count(), want_accum=True)
    assert np.array_equal(a, b) and np.array_equal(_bits(fa), _bits(fb))
    assert sa["segments"] == sb["segments"]
    assert 0 < sb["render_ms"] <= sb["frame_ms"] <= sb["total_ms"]
    assert 0 < sa["render_ms"] <= sa["frame_ms"] <= sa["total_ms"]
    # every communicator of the clique reports the whole clique (ncclCommCount)
    info = rt.last_multi_info()
    n = rt.device_count()
    assert info == {"path": "rccl", "devices": n, "comm_ranks": [n] * n}


def test_entry_points_restore_current_device(gpu_available):
    """rtc_render(device=k), rtc_render_multi and a device-resident launch leave the caller's (and torch's)
    current device where it was (the library used to leave the render's device current)."""
    import torch

    tris, _ = load_tris("complex")
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(32, 18, 2, 10, True)
    last = rt.device_count() - 1
    torch.cuda.set_device(last)
    rt.render(tris, None, scene, cam, cfg, device=0)
    assert torch.cuda.current_device() == last
    rt.render_multi(tris, None, scene, cam, cfg, rt.device_count())
    assert torch.cuda.current_device() == last
    ds = rt.DeviceScene(tris, None, device=0)
    assert torch.cuda.current_device() == last
    out = torch.zeros((18, 32, 3), dtype=torch.uint8, device="cuda:0")
    ds.render_rows_async(scene, cam, cfg, out.data_ptr(), stream=torch.cuda.current_stream(0).cuda_stream)
    torch.cuda.synchronize(0)
    assert torch.cuda.current_device() == last
    ds.close()
    torch.cuda.set_device(0)


def test_cli_multi_gpu_flag_uses_rccl_path(tmp_path, gpu_available):
    """The drop-in CLI's --gpus N (rtc_render_multi, RCCL) writes the reference's BMP byte for byte."""
    g = GOLD["ultracomplex_160x90x4"]
    tris, _ = load_tris("ultracomplex")
    obj = tmp_path / "scene.obj"
    _write_obj_from_tris(obj, tris)
    r = subprocess.run([rt.CLI_PATH, "-i", str(obj), "-s", "160", "90", "--spp", "4", "--gpus",
                        str(rt.device_count()), "--stats", "-o", str(tmp_path / "o.bmp")], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert hashlib.md5((tmp_path / "o.bmp").read_bytes()).hexdigest() == g["bmp_md5"]


def test_full_size_properties(gpu_available):
    """The BASELINE workload (ultracomplex 1920x1080x64): deterministic, hoisting bit-exact, and a row sample
    of the frame matches the oracle bit for bit with identical paths."""
    tris, tonly = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(1920, 1080, 64, 10, True)
    c1, a1, s1 = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    c2, a2, s2 = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a2)) and s1["segments"] == s2["segments"]
    c3, a3, s3 = rt.render(tris, None, scene, cam, rt.RenderConfig(1920, 1080, 64, 10, True, hoist=True),
                           want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a3))
    # 1.0317 segments / sample at 480x270 (same scene, same camera)
    assert 1.02 < s1["segments"] / s1["samples"] < 1.045
    # row sample vs oracle, bit for bit (floats and u8): rows y = 5 + 48k (23 rows, 2.8 M samples)
    d = RtcRenderDesc(1920, 1080, 64, 10, tonly, 5, 48, 0)
    ocol, oacc, oseg = orc.render(tris, None, scene, cam, d, threads=16)
    mx, over, exact = _compare(a1[5::48], oacc)
    print(f"1080p x64 row sample: max|d|={mx:.3g} over={over} exact={exact:.5f}")
    assert np.array_equal(_bits(a1[5::48]), _bits(oacc)) and np.array_equal(c1[5::48], ocol)
    # the same rows rendered alone take the oracle's paths
    _, _, sr = rt.render(tris, None, scene, cam, rt.RenderConfig(1920, 1080, 64, 10, True, row_start=5, row_stride=48))
    assert sr["segments"] == oseg


@pytest.mark.parametrize("scene,W,H,spp,row0,stride", [("cube", 1920, 1080, 16, 3, 24),
                                                        ("fsuzane", 1920, 1080, 64, 7, 40)])
def test_full_size_baseline_configs(scene, W, H, spp, row0, stride, gpu_available):
    """BASELINE.json C2 (cube.obj 1920x1080x16) and C3 (fsuzane.obj 1920x1080x64) at full size on one GPU:
    deterministic, and a row sample (rows y = row0 + k*stride) matches the oracle bit for bit with identical
    paths."""
    tris, tonly = load_tris(scene)
    sc, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(W, H, spp, 10, True)
    c1, a1, s1 = rt.render(tris, None, sc, cam, cfg, want_accum=True)
    c2, a2, s2 = rt.render(tris, None, sc, cam, cfg, want_accum=True)
    assert np.array_equal(_bits(a1), _bits(a2)) and s1["segments"] == s2["segments"]
    d = RtcRenderDesc(W, H, spp, 10, tonly, row0, stride, 0)
    ocol, oacc, oseg = orc.render(tris, None, sc, cam, d, threads=16)
    assert np.array_equal(_bits(a1[row0::stride]), _bits(oacc)) and np.array_equal(c1[row0::stride], ocol)
    # the same rows rendered alone on the GPU take the same paths as on the CPU
    cr, ar, sr = rt.render(tris, None, sc, cam, rt.RenderConfig(W, H, spp, 10, True, row_start=row0, row_stride=stride),
                           want_accum=True)
    assert np.array_equal(_bits(ar), _bits(oacc)) and sr["segments"] == oseg
    print(f"{scene} {W}x{H}x{spp}: frame {s1['frame_ms']:.3f} ms (render {s1['render_ms']:.3f} ms)")


@pytest.mark.parametrize("scene,spp", [("ultracomplex", 64), ("complex", 64), ("ultracomplex", 256)])
def test_full_size_4k_configs(scene, spp, gpu_available):
    """BASELINE.json at 3840x2160 -- NS (ultracomplex x64), C4 (complex x64), C5 (ultracomplex x256) -- rendered
    whole on one GPU (the tile cones, chain windows and deferred slots at 4K sizes; main.c:246 needs a 1 GiB stack
    for this frame on the CPU): a row sample y = 3 + 90k (24 rows) equals the oracle bit for bit, floats and u8,
    and the same rows rendered alone take the oracle's paths (equal segment counts)."""
    tris, tonly = load_tris(scene)
    sc, cam, _ = setup_from_flags({})
    W, H, row0, stride = 3840, 2160, 3, 90
    c1, a1, s1 = rt.render(tris, None, sc, cam, rt.RenderConfig(W, H, spp, 10, True), want_accum=True)
    d = RtcRenderDesc(W, H, spp, 10, tonly, row0, stride, 0)
    ocol, oacc, oseg = orc.render(tris, None, sc, cam, d, threads=16)
    assert oacc.shape[0] == 24
    mx, over, exact = _compare(a1[row0::stride], oacc)
    print(f"{scene} {W}x{H}x{spp}: frame {s1['frame_ms']:.3f} ms; row sample max|d|={mx:.3g} exact={exact:.6f}")
    assert np.array_equal(_bits(a1[row0::stride]), _bits(oacc)) and np.array_equal(c1[row0::stride], ocol)
    _, _, sr = rt.render(tris, None, sc, cam, rt.RenderConfig(W, H, spp, 10, True, row_start=row0, row_stride=stride))
    assert sr["segments"] == oseg
    # the whole frame takes the survey's path statistics (~1.03 segments per sample)
    assert 1.0 < s1["segments"] / s1["samples"] < 1.05


@pytest.mark.parametrize("W,H", [(1920, 1080), (3840, 2160)], ids=["headline_1080p64", "ns_4k64"])
def test_whole_frame_bit_exact(W, H, gpu_available):
    """the ENTIRE metric frame (ultracomplex 1920x1080x64, BASELINE.json `metric`) and the entire NS
    frame (3840x2160x64) against the CPU oracle rendering every row (oracle/rtc_oracle.c, bit-identical to the
    reference's own build on every golden fixture): float accumulator bits, Color[] bytes and the traced segment count,
    all equal.  The frame the bench times (pipelined RTC_F_OVERLAP launches on the cull streams, in-kernel sums) is
    compared too, byte for byte (main.c:81-104)."""
    import torch

    tris, tonly = load_tris("ultracomplex")
    sc, cam, _ = setup_from_flags({})
    spp = 64
    c1, a1, s1 = rt.render(tris, None, sc, cam, rt.RenderConfig(W, H, spp, 10, True), want_accum=True)
    ocol, oacc, oseg = orc.render(tris, None, sc, cam, RtcRenderDesc(W, H, spp, 10, tonly, 0, 1, 0), threads=16)
    assert oacc.shape == (H, W, 3)
    mx, over, exact = _compare(a1, oacc)
    print(f"ultracomplex {W}x{H}x{spp} whole frame: max|d|={mx:.3g} over={over} exact={exact:.7f} "
          f"segments {s1['segments']} vs {oseg}")
    assert np.array_equal(_bits(a1), _bits(oacc))
    assert np.array_equal(c1, ocol)
    assert s1["segments"] == oseg
    # the benchmarked launch path: three pipelined frames into three buffers, each equal to the oracle's bytes
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    bufs = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    for b in bufs:
        ds.render_rows_async(sc, cam, rt.RenderConfig(W, H, spp, 10, True, overlap=True), b.data_ptr(),
                             stream=st.cuda_stream)
    torch.cuda.synchronize()
    for b in bufs:
        assert np.array_equal(b.cpu().numpy(), ocol)
    ds.close()


def test_overlapped_then_other_launches_same_buffer(gpu_available):
    """an RTC_F_OVERLAP launch leaves its sky pass running on the side stream.  A following launch
    that is not overlapped -- a joined split launch, a brute-force (no tile cull) launch, a debug launch -- must
    not race it: the overlapped frame with camera A, then each of those with camera B into the SAME buffer,
    equals rtc_render of camera B bit for bit (a stale sky pass of camera A would leave its values behind)."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene = rt.default_scene()
    cam_a = rt.camera_basis()
    cam_b = rt.camera_basis((-4.0, -1.9, -5.2), (0.6, -1.0, 1.3), 1.1)
    W, H, spp = 640, 360, 32  # a sky pass long enough to still run when the next launch is enqueued
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    for follow in ({}, {"tile_cull": False}, {"coop": False}, {"debug_bounces": True}, {"hoist": True}):
        cfg_b = rt.RenderConfig(W, H, spp, 10, True, **follow)
        ref_b, _, _ = rt.render(tris, None, scene, cam_b, cfg_b)
        for _ in range(3):
            ds.render_rows_async(scene, cam_a, rt.RenderConfig(W, H, spp, 10, True, overlap=True), buf.data_ptr(),
                                 stream=st.cuda_stream)
            ds.render_rows_async(scene, cam_b, cfg_b, buf.data_ptr(), stream=st.cuda_stream)
            st.synchronize()  # the follower joined (or waited for) every pass it depends on: its stream suffices
            assert np.array_equal(buf.cpu().numpy(), ref_b), follow
    ds.close()


def test_frame_event_is_one_shot(gpu_available):
    """rtc_scene_set_frame_event / _geometry_event arm an event for the next launch only (a launch used
    to record a released event): arm, launch, release the events, launch again (overlapped and joined) -- no
    crash, every frame right; and a launch after the armed one does not record it again."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H, spp = 1920, 1080, 64
    ref, _, _ = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    for overlap in (True, False):
        cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=overlap)
        ev, geo = torch.cuda.Event(), torch.cuda.Event()
        ev.record(st)
        geo.record(st)
        ds.set_frame_event(ev.cuda_event)
        ds.set_geometry_event(geo.cuda_event)
        ds.render_rows_async(scene, cam, cfg, buf.data_ptr(), stream=st.cuda_stream)
        ev.synchronize()
        assert np.array_equal(buf.cpu().numpy(), ref)
        # the next launch (a ~0.5 ms frame) does not record ev: it stays complete while that launch runs
        ds.render_rows_async(scene, cam, cfg, buf.data_ptr(), stream=st.cuda_stream)
        assert ev.query()
        torch.cuda.synchronize()
        del ev, geo  # hipEventDestroy
        torch.cuda.synchronize()
        for _ in range(3):
            ds.render_rows_async(scene, cam, cfg, buf.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), ref)
    ds.close()


@pytest.mark.parametrize("name", ["suzannes_96x54x4", "suzannes_cam_64x48x2"])
def test_large_scene(name, gpu_available):
    """suzannes.obj (5,208 triangles = 651 clusters in 21 chunks: rtc_render_chain with records from global
    memory and chunk-level culling) against the reference's golden hash; == the one-lane-per-pixel kernel with
    and without tile culling, bit for bit, with the same segment counts."""
    g = GOLD[name]
    tris, tonly = load_tris(g["scene"])
    assert len(tris) > 256
    scene, cam, mb = setup_from_flags(g["flags"])
    base = rt.RenderConfig(g["width"], g["height"], g["spp"], mb, bool(tonly))
    c1, a1, s1 = rt.render(tris, None, scene, cam, base, want_accum=True)
    assert hashlib.sha256(a1.tobytes()).hexdigest() == g["float_sha256"]
    for kw in ({"tile_cull": False}, {"coop": False}, {"chain_inline": True}, {"hoist": True}):
        c0, a0, s0 = rt.render(tris, None, scene, cam, rt.RenderConfig(**{**base.__dict__, **kw}), want_accum=True)
        assert np.array_equal(_bits(a0), _bits(a1)) and np.array_equal(c0, c1) and s0["segments"] == s1["segments"], kw


def test_large_scene_full_frame(gpu_available):
    """suzannes.obj at 640x360x16 through rtc_render_chain vs the oracle on a row sample, bit for bit."""
    tris, tonly = load_tris("suzannes")
    scene, cam, _ = setup_from_flags({})
    W, H, spp = 640, 360, 16
    c1, a1, s1 = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True), want_accum=True)
    d = RtcRenderDesc(W, H, spp, 10, tonly, 1, 9, 0)
    ocol, oacc, oseg = orc.render(tris, None, scene, cam, d, threads=16)
    assert np.array_equal(_bits(a1[1::9]), _bits(oacc)) and np.array_equal(c1[1::9], ocol)
    print(f"suzannes {W}x{H}x{spp}: render {s1['render_ms']:.3f} ms")


def test_edge_sizes(gpu_available):
    tris, tonly = load_tris("fsuzane")
    scene, cam, _ = setup_from_flags({})
    for (w, h, spp, mb) in [(1, 1, 3, 10), (2, 1, 1, 10), (1, 3, 2, 1), (17, 9, 0, 10), (17, 9, 2, 0), (255, 3, 1, 10)]:
        col, acc, st = rt.render(tris, None, scene, cam, rt.RenderConfig(w, h, spp, mb, True), want_accum=True)
        ocol, oacc, oseg = orc.render(tris, None, scene, cam, RtcRenderDesc(w, h, spp, mb, tonly, 0, 1, 0), threads=2)
        mx, over, _ = _compare(acc, oacc)
        assert over == 0 and st["segments"] == oseg, (w, h, spp, mb)


def _write_obj_from_tris(path, tris):
    """An OBJ (+ MTL) whose loadOBJTriangles result is `tris` byte for byte (tools/obj_export.py)."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from obj_export import write_obj

    write_obj(str(path), tris)


@pytest.mark.parametrize("name", ["cube_64x36x4", "C1_simplest_256x256x1"])
def test_cli_bmp_matches_reference(name, tmp_path, gpu_available):
    """The drop-in CLI (flag-compatible with main.c) writes the reference's BMP byte for byte."""
    g = GOLD[name]
    tris, _ = load_tris(g["scene"])
    obj = tmp_path / "scene.obj"
    _write_obj_from_tris(obj, tris)
    assert rt.loadOBJTriangles(str(obj)).tobytes() == tris.tobytes()
    r = subprocess.run([rt.CLI_PATH, "-i", str(obj), "-s", str(g["width"]), str(g["height"]), "--spp", str(g["spp"]),
                        "-o", str(tmp_path / "o.bmp")], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert hashlib.md5((tmp_path / "o.bmp").read_bytes()).hexdigest() == g["bmp_md5"]


@pytest.mark.parametrize("nbytes", [1, 15, 4096, 1920 * 1080 * 3 + 7])
def test_frame_copies(nbytes, gpu_available):
    """rtc_copy_async (a few workgroups, 16-byte words + byte tail) and rtc_copy_d2h_dma (SDMA engines) deliver
    the device bytes into pinned host memory exactly."""
    import torch

    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    ref = src.cpu()
    h1 = torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)
    h2 = torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.current_stream()
    rt.copy_async(h1.data_ptr(), src.data_ptr(), nbytes, 32, st.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(h1, ref)
    rt.copy_d2h_dma(h2.data_ptr(), src.data_ptr(), nbytes)
    assert torch.equal(h2, ref)


def _shm_frame(nbytes):
    """A host frame in POSIX shared memory (what the ranks of a multi-process job all map), page-locked."""
    import mmap

    fd = os.open(f"/dev/shm/rtc_test_{os.getpid()}", os.O_CREAT | os.O_RDWR, 0o600)
    os.ftruncate(fd, nbytes)
    mm = mmap.mmap(fd, nbytes)
    os.close(fd)
    os.unlink(f"/dev/shm/rtc_test_{os.getpid()}")
    arr = np.frombuffer(mm, np.uint8)
    rt.host_register(arr.ctypes.data, nbytes)
    return mm, arr


@pytest.mark.parametrize("band", [1, 8])
@pytest.mark.parametrize("W,H", [(1920, 1080), (121, 67)])
def test_strided_row_copies_build_host_frame(W, H, band, gpu_available):
    """The multi-GPU host-frame path: ranks' compact rows y = r + k*G (G = 2..8 simulated on one device), each
    copied by rtc_copy_rows_d2h_dma straight into its places of one host frame (pitch G*W*3; SDMA sub-window copy,
    or per-row copies when W*3 is not a multiple of 4) -- into hipHostMalloc'd memory and into a registered
    shared-memory frame -- equal the single-GPU host frame byte for byte (main.c:84, :285-302)."""
    import torch

    from raytracingc_amd.distributed import copy_rank_rows_to_host, rank_config, rows_per_rank

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(W, H, 4, 10, True)
    ref, _, _ = rt.render(tris, None, scene, cam, cfg)
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.current_stream()
    mm, shm = _shm_frame(H * W * 3)
    try:
        for G in (2, 3, 4, 8):
            rows = rows_per_rank(H, G, band)
            parts = torch.zeros((G, rows, W, 3), dtype=torch.uint8, device="cuda")
            for r in range(G):
                rc = rank_config(cfg, r, G, band)
                if rc.rows():
                    ds.render_rows_async(scene, cam, rc, parts[r].data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize()
            pinned = torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True)
            shm[:] = 0
            for r in range(G):
                for dst in (pinned.data_ptr(), shm.ctypes.data):
                    copy_rank_rows_to_host(dst, W, H, r, G, parts[r].data_ptr(), band)
            assert np.array_equal(pinned.numpy(), ref), f"G={G} pinned"
            assert np.array_equal(shm.reshape(H, W, 3), ref), f"G={G} shm"
    finally:
        rt.host_unregister(shm.ctypes.data)
        del shm
        mm.close()
        ds.close()


@pytest.mark.parametrize("band", [0, 8])
@pytest.mark.parametrize("name", ["complex", "ultracomplex"])
def test_render_multi_host_rows_equals_render(name, band, gpu_available):
    """rtc_render_multi with RTC_F_HOST_ROWS (no gather: every device copies its rows -- or bands of 8 rows -- into the
    host frame) == rtc_render bit for bit, colors and floats, same paths."""
    tris, tonly = load_tris(name)
    scene, cam, _ = setup_from_flags({})
    cfg = rt.RenderConfig(160, 90, 8, 10, True)
    a, fa, sa = rt.render(tris, None, scene, cam, cfg, want_accum=True)
    b, fb, sb = rt.render_multi(tris, None, scene, cam,
                                rt.RenderConfig(160, 90, 8, 10, True, host_rows=True, row_band=band),
                                rt.device_count(), want_accum=True)
    assert np.array_equal(a, b) and np.array_equal(_bits(fa), _bits(fb))
    assert sa["segments"] == sb["segments"]
    assert 0 < sb["render_ms"] <= sb["frame_ms"] <= sb["total_ms"]
    assert rt.last_multi_info() == {"path": "host_rows", "devices": rt.device_count(), "comm_ranks": []}


def test_frame_loop_pipelined_host_frames(gpu_available):
    """rtc_frame_loop (native pipelined frames: RTC_F_OVERLAP renders, a copy thread moving each frame's rows into
    host memory with the SDMA engines): every buffer's host frame equals rtc_render's, for the whole frame and for
    the interleaved rows of G = 3 "ranks" written into one shared host frame."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H, spp = 640, 360, 16
    ref, _, _ = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    host = [torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    out = ds.frame_loop(scene, cam, rt.RenderConfig(W, H, spp, 10, True), [d.data_ptr() for d in dev],
                        [h.data_ptr() for h in host], W * 3, 7, st.cuda_stream)
    assert out["frames"] == 7 and out["wall_ms"] > 0 and out["copy_ms_median"] > 0
    for h in host:
        assert np.array_equal(h.numpy(), ref)
    G = 3
    from raytracingc_amd.distributed import rank_config

    mm, shm = _shm_frame(2 * H * W * 3)
    try:
        frames = shm.reshape(2, H, W, 3)
        for band in (1, 8):  # single rows, then bands of 8 rows (360 = 45 bands: a rank's last band may be cut)
            shm[:] = 0
            for r in range(G):
                cfg = rank_config(rt.RenderConfig(W, H, spp, 10, True), r, G, band)
                ds.frame_loop(scene, cam, cfg, [d.data_ptr() for d in dev[:2]],
                              [frames[b].ctypes.data + r * band * W * 3 for b in range(2)], G * band * W * 3, 4,
                              st.cuda_stream)
            for b in range(2):
                assert np.array_equal(frames[b], ref), f"buffer {b} band {band}"
    finally:
        rt.host_unregister(shm.ctypes.data)
        del frames, shm
        mm.close()
    ds.close()


@pytest.mark.parametrize("band", [1, 8])
@pytest.mark.parametrize("scene,spp,G", [("complex", 64, 4), ("ultracomplex", 64, 8), ("ultracomplex", 256, 8)])
def test_4k_row_shares_assemble_bit_exact(scene, spp, G, band, gpu_available):
    """BASELINE.json C4 (complex 3840x2160x64 over 4 GPUs), NS (ultracomplex 4K x64) and C5 (ultracomplex 4K x256)
    over 8 GPUs: every rank's share (rows y = r + k*G, main.c:84 lifted to GPUs, or the bands r + k*G of 8 rows:
    north_star's row-tile split; 540 / 270 rows of 3840, so the deferred-sum path) rendered on one device, assembled
    two ways -- the RCCL path's re-interleave on the device (rtc_deinterleave_async / _bands_async) and the host-frame
    path's strided SDMA copies into one pinned frame (rtc_copy_rows_d2h_dma) -- equals the single-GPU 4K frame bit for
    bit, bytes and floats; the last share equals the oracle's render of the same rows bit for bit with the same
    paths; and the pipelined per-rank frame loop the bench runs (rtc_frame_loop, RTC_F_OVERLAP) builds the same
    host frame."""
    import torch

    from raytracingc_amd.distributed import band_rows, copy_rank_rows_to_host, rank_config, rows_per_rank

    tris, tonly = load_tris(scene)
    sc, cam, _ = setup_from_flags({})
    W, H = 3840, 2160
    full = rt.RenderConfig(W, H, spp, 10, True)
    ref, racc, _ = rt.render(tris, None, sc, cam, full, want_accum=True)
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.current_stream().cuda_stream
    rows = rows_per_rank(H, G, band)
    parts = torch.zeros((G, rows, W, 3), dtype=torch.uint8, device="cuda")
    accs = torch.zeros((G, rows, W, 3), dtype=torch.float32, device="cuda")
    for r in range(G):
        cfg = rank_config(full, r, G, band)
        assert cfg.rows() * W > 600000  # not a small share: deferred sums (rtc_accumulate_samples)
        ds.render_rows_async(sc, cam, cfg, parts[r].data_ptr(), accs[r].data_ptr(), None, st)
    out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    rt.deinterleave_async(parts.data_ptr(), G, rows, W, H, out.data_ptr(), st, band)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref), "device re-interleave"
    pinned = torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True)
    for r in range(G):
        copy_rank_rows_to_host(pinned.data_ptr(), W, H, r, G, parts[r].data_ptr(), band)
    assert np.array_equal(pinned.numpy(), ref), "strided SDMA host frame"
    a = accs.cpu().numpy()
    for r in range(G):
        ys = band_rows(H, r, G, band)
        assert np.array_equal(_bits(a[r, :len(ys)]), _bits(racc[ys])), f"rank {r} floats"
    # the pipelined per-rank loop of bench.py, every rank's frames into one pinned host frame pair
    host = [torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    dev = [torch.zeros((rows, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    lst = torch.cuda.Stream()
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    for r in range(G):
        cfg = rank_config(full, r, G, band)
        ds.frame_loop(sc, cam, cfg, [d.data_ptr() for d in dev], [h.data_ptr() + r * band * W * 3 for h in host],
                      G * band * W * 3, 3, lst.cuda_stream)
    for h in host:
        assert np.array_equal(h.numpy(), ref), "frame loop host frame"
    ds.close()
    r0 = G - 1
    rc = rank_config(full, r0, G, band)
    ocol, oacc, oseg = orc.render(tris, None, sc, cam, rc.desc(), threads=16)
    n = rc.rows()
    assert n == len(band_rows(H, r0, G, band)) == oacc.shape[0]
    assert np.array_equal(_bits(a[r0, :n]), _bits(oacc)) and np.array_equal(parts[r0, :n].cpu().numpy(), ocol)
    _, _, sr = rt.render(tris, None, sc, cam, rc)
    assert sr["segments"] == oseg


def test_prep_skip_across_streams(gpu_available):
    """rtc_prep_primary is skipped when the camera origin and the stream are those of the previous split
    launch, whose tile cull zeroed this launch's sub-list counters.  Same origin on streams A, B, A, A (joined and
    pipelined), then a camera change and back: every frame equals rtc_render bit for bit."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene = rt.default_scene()
    cam, cam2 = rt.camera_basis(), rt.camera_basis((-4.0, -1.9, -5.2), (0.6, -1.0, 1.3), 1.1)
    W, H, spp = 256, 144, 8
    ref = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))[0]
    ref2 = rt.render(tris, None, scene, cam2, rt.RenderConfig(W, H, spp, 10, True))[0]
    ds = rt.DeviceScene(tris, None)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for overlap in (False, True):
        cfg = rt.RenderConfig(W, H, spp, 10, True, overlap=overlap)
        for s, c, want in ((sa, cam, ref), (sb, cam, ref), (sa, cam, ref), (sa, cam, ref), (sa, cam2, ref2),
                           (sb, cam2, ref2), (sa, cam, ref)):
            buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
            ev = torch.cuda.Event()
            ev.record(s)
            ds.set_frame_event(ev.cuda_event)
            ds.render_rows_async(scene, c, cfg, buf.data_ptr(), stream=s.cuda_stream)
            ev.synchronize()
            assert np.array_equal(buf.cpu().numpy(), want), overlap
    torch.cuda.synchronize()
    ds.close()


def test_moving_camera_frame_loop(gpu_available):
    """rtc_frame_loop_cameras (the bench's moving-camera leg): frame k renders with camera k mod 5 into buffer
    k mod 3; each host buffer holds the last frame written into it, equal to rtc_render of that frame's camera."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene = rt.default_scene()
    cams = [rt.camera_basis((-4.75 + 0.3 * k, -1.5 - 0.05 * k, -4.75 + 0.2 * k), rt.DEFAULT_LOOKING_AT, 1.0)
            for k in range(5)]
    W, H, spp, frames = 320, 180, 8, 7
    refs = [rt.render(tris, None, scene, c, rt.RenderConfig(W, H, spp, 10, True))[0] for c in cams]
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    dev = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    host = [torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    out = ds.frame_loop(scene, cams, rt.RenderConfig(W, H, spp, 10, True), [d.data_ptr() for d in dev],
                        [h.data_ptr() for h in host], W * 3, frames, st.cuda_stream)
    assert out["frames"] == frames
    for b in range(3):
        k = max(k for k in range(frames) if k % 3 == b)
        assert np.array_equal(host[b].numpy(), refs[k % 5]), f"buffer {b} (frame {k})"
    ds.close()


def test_empty_launch_consumes_frame_event(gpu_available):
    """a launch that selects no rows returns at once but still takes (and records) the armed one-shot
    events, so the next launch cannot record an event its caller released after the empty one."""
    import torch

    tris, _ = load_tris("ultracomplex")
    scene, cam, _ = setup_from_flags({})
    W, H, spp = 160, 90, 4
    ref = rt.render(tris, None, scene, cam, rt.RenderConfig(W, H, spp, 10, True))[0]
    ds = rt.DeviceScene(tris, None)
    st = torch.cuda.Stream()
    buf = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # (the zero fills ran on the current stream, not the launch stream)
    ev = torch.cuda.Event()
    ev.record(st)
    ds.set_frame_event(ev.cuda_event)
    ds.render_rows_async(scene, cam, rt.RenderConfig(W, H, spp, 10, True, row_start=H), buf.data_ptr(),
                         stream=st.cuda_stream)
    ev.synchronize()
    del ev
    torch.cuda.synchronize()
    for overlap in (False, True):
        ds.render_rows_async(scene, cam, rt.RenderConfig(W, H, spp, 10, True, overlap=overlap), buf.data_ptr(),
                             stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), ref)
    ds.close()

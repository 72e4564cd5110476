"""The sky kernel's per-pixel sun skip (rtc_device.h sun_vanishes / env_vanish_limit, round 6).

Where focus * log2(x) lies below the scene's limit the sun term of getEnvironmentLight (raytracing.c:155-158) is below half
an ulp of every colour component, so skipping it leaves the reference's value bit for bit.  CPU: the limit the library
computes (host code) against its definition, and the claim itself against the oracle's environment -- every ray the
limit admits gives the same bits as the environment without a sun.  GPU: the device's flags and the environment evaluated
with them equal the oracle's on every ray (boundary rays included)."""
from __future__ import annotations

import math
import zlib

import numpy as np
import pytest

import oracle.binding as orc
import raytracingc_amd as rt
from raytracingc_amd._abi import RAY_DT, SCENE_DT


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _scene(sun, horizon, zenith, ground, focus, intensity):
    s = np.zeros(1, SCENE_DT)
    sun = np.asarray(sun, np.float64)
    sun = (sun / np.linalg.norm(sun)).astype(np.float32)
    for k, v in (("normalizedSunDirection", sun), ("skyColorHorizon", horizon), ("skyColorZenith", zenith),
                 ("groundColor", ground)):
        s[k]["x"], s[k]["y"], s[k]["z"] = v
    s["sunFocus"], s["sunIntensity"] = focus, intensity
    return s[0]


def _limit_py(s):
    """env_vanish_limit restated: H = 2^(floor(log2(m (1 - 2^-20))) - 24), limit = log2(H / intensity) - 1e-5."""
    f, i = float(s["sunFocus"]), float(s["sunIntensity"])
    cols = [float(s[k][c]) for k in ("groundColor", "skyColorHorizon", "skyColorZenith") for c in "xyz"]
    if not (0 < f < 3.0e38 and 0 < i < 3.0e38) or not all(2.0 ** -60 <= c <= 2.0 ** 60 for c in cols):
        return -math.inf
    e = math.floor(math.log2(min(cols) * (1 - 2.0 ** -20)))
    return math.log2(2.0 ** (e - 24) / i) - 1e-5


def _scenes():
    d = rt.default_scene()
    yield "default", np.frombuffer(bytes(d), SCENE_DT)[0].copy()
    rng = np.random.default_rng(7)
    for k in range(10):
        cols = rng.uniform(0.02, 1.5, (3, 3)).astype(np.float32)
        if k % 3 == 0:  # a colour exactly at a power of two: the exponent bound at its tightest
            cols[rng.integers(3), rng.integers(3)] = 2.0 ** -int(rng.integers(1, 5))
        sun = rng.normal(size=3)
        sun[1] = -abs(sun[1])
        yield f"r{k}", _scene(sun, cols[0], cols[1], cols[2], float(rng.choice([4.0, 22.0, 100.0, 700.0])),
                              float(rng.choice([0.75, 3.0, 40.0, 0.01])))
    yield "zero_colour", _scene((0, -1, 0), (1, 1, 1), (0.3, 0.9, 0.0), (0.6, 0.6, 0.6), 22.0, 0.75)
    yield "neg_intensity", _scene((0, -1, 0), (1, 1, 1), (0.3, 0.9, 0.8), (0.6, 0.6, 0.6), 22.0, -0.75)
    yield "zero_focus", _scene((0, -1, 0), (1, 1, 1), (0.3, 0.9, 0.8), (0.6, 0.6, 0.6), 0.0, 0.75)


def _rays(s, n, rng, lim):
    """Directions above the horizon (dir.y < 0 is the sun's side, raytracing.c:156) at random, plus directions whose
    focus * log2(x) lies within 0.05 of the limit (the boundary where the skip is tightest)."""
    sun = np.array([s["normalizedSunDirection"][c] for c in "xyz"], np.float64)
    d = rng.normal(size=(n, 3))
    if np.isfinite(lim):
        m = n // 2
        x = 2.0 ** ((lim + rng.uniform(-0.05, 0.01, m)) / float(s["sunFocus"]))
        x = np.clip(x, 1e-30, 1.0)
        p = rng.normal(size=(m, 3))
        p -= (p @ sun)[:, None] * sun
        p /= np.linalg.norm(p, axis=1)[:, None]
        d[:m] = x[:, None] * sun + np.sqrt(1 - x * x)[:, None] * p
    d /= np.linalg.norm(d, axis=1)[:, None]
    r = np.zeros(n, RAY_DT)
    r["dir"]["x"], r["dir"]["y"], r["dir"]["z"] = d.astype(np.float32).T
    return r


def test_limit_matches_definition():
    for name, s in _scenes():
        lim = rt.env_vanish_limit(s)
        want = _limit_py(s)
        if math.isinf(want):
            assert lim == want, name
        else:
            assert abs(lim - want) < 1e-12, name
    d = np.frombuffer(bytes(rt.default_scene()), SCENE_DT)[0]
    # the headline scene: m = 0.263 -> H = 2^-26; skipped where 22 log2(x) < log2(2^-26 / 0.75), x < ~0.447
    assert abs(rt.env_vanish_limit(d) - (math.log2(2.0 ** -26 / 0.75) - 1e-5)) < 1e-12


@pytest.mark.parametrize("name,s", list(_scenes()), ids=lambda v: v if isinstance(v, str) else "")
def test_skip_leaves_oracle_value(name, s):
    """Every ray the limit admits (with a margin for numpy's log2 against glibc's) has the oracle's environment equal to
    the same environment without a sun (intensity +0: sun term +0), bit for bit."""
    lim = rt.env_vanish_limit(s)
    if not np.isfinite(lim):
        return
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    rays = _rays(s, 20000, rng, lim)
    d = np.stack([rays["dir"][c] for c in "xyz"], 1).astype(np.float32)
    sun = np.array([s["normalizedSunDirection"][c] for c in "xyz"], np.float32)
    x = (d[:, 0] * sun[0] + d[:, 1] * sun[1]) + d[:, 2] * sun[2]
    ok = (d[:, 1] < 0) & (x >= 2.0 ** -126) & (x < 1)
    ylogx = np.full(len(x), np.inf)
    ylogx[ok] = float(s["sunFocus"]) * np.log2(x[ok].astype(np.float64))
    adm = ylogx < lim - 1e-9 * max(1.0, float(s["sunFocus"]))
    assert adm.sum() > 100
    nosun = s.copy()
    nosun["sunIntensity"] = 0.0
    a = orc.environment(rays[adm], np.repeat(s[None], adm.sum()))
    b = orc.environment(rays[adm], np.repeat(nosun[None], adm.sum()))
    assert np.array_equal(_bits(a), _bits(b))


@pytest.mark.gpu
@pytest.mark.parametrize("name,s", list(_scenes()), ids=lambda v: v if isinstance(v, str) else "")
def test_device_skip_bit_exact(name, s, gpu_available):
    lim = rt.env_vanish_limit(s)
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    rays = _rays(s, 40000, rng, lim)
    sc = np.repeat(s[None], len(rays))
    v, out = rt.sun_vanish_probe(rays, sc)
    ref = orc.environment(rays, sc)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(out), nan)
    assert np.array_equal(_bits(out[~nan]), _bits(ref[~nan]))
    if np.isfinite(lim):
        assert 100 < v.sum() < len(v)
    else:
        assert v.sum() == 0

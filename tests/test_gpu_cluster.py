"""Soundness of the bounce-ray cluster culling (DevCluster / cluster_culled in rtc_render.hip).

A bounce ray of the cooperative path skips a cluster of 8 triangles when its half-line provably passes
farther from the cluster's bounding ball than any hit rayTriangle (raytracing.c:186-214) could report.  If
the bound were wrong, a pixel would differ from the reference only for rare grazing rays, which the
frame-level parity tests could miss; this test aims millions of rays at exactly those cases -- from points
on the triangles (as bounce rays start), at other triangles' vertices, edges and planes, at grazing angles
near the |det| = EPSILON threshold, in scaled copies of the scenes -- and requires that no triangle inside
a culled cluster is ever hit.  The per-ray test runs the same device functions the renderer uses."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import load_tris

import raytracingc_amd as rt
from raytracingc_amd._abi import RAY_DT

pytestmark = pytest.mark.gpu


def _verts(t):
    return (np.stack([t["posA"][c] for c in "xyz"], 1).astype(np.float64),
            np.stack([t["posB"][c] for c in "xyz"], 1).astype(np.float64),
            np.stack([t["posC"][c] for c in "xyz"], 1).astype(np.float64),
            np.stack([t["normal"][c] for c in "xyz"], 1).astype(np.float64))


def _unit(v):
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def _bounce_like_rays(tris, n, rng):
    """Origins on random triangles, directions as calcColor forms them (raytracing.c:276-280): a lerp of
    normalize(N + random unit) and a reflection, by a random smoothness (so |dir| < 1 too)."""
    A, B, C, N = _verts(tris)
    k = rng.integers(0, len(tris), n)
    u, v = rng.random(n), rng.random(n)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    pos = A[k] + u[:, None] * (B[k] - A[k]) + v[:, None] * (C[k] - A[k])
    diffuse = _unit(N[k] + _unit(rng.normal(size=(n, 3))))
    incoming = _unit(rng.normal(size=(n, 3)))
    spec = incoming - 2 * np.sum(incoming * N[k], 1, keepdims=True) * N[k]
    s = rng.random(n)[:, None]
    return pos, diffuse * (1 - s) + spec * s


def _aimed_rays(tris, n, rng):
    """Origins on triangles, aimed at vertices / edge points / interior points of other triangles, with
    small perturbations: hits and near misses right at the bounding balls' boundaries."""
    A, B, C, N = _verts(tris)
    pos, _ = _bounce_like_rays(tris, n, rng)
    j = rng.integers(0, len(tris), n)
    w = rng.dirichlet([0.3, 0.3, 0.3], n)
    target = w[:, :1] * A[j] + w[:, 1:2] * B[j] + w[:, 2:] * C[j]
    d = target - pos
    scale = np.linalg.norm(d, axis=1, keepdims=True) + 1e-30
    d = d / scale + rng.normal(size=(n, 3)) * (10.0 ** rng.uniform(-7, -1, (n, 1)))
    return pos, d


def _grazing_rays(tris, n, rng):
    """Directions almost in the plane of a random target triangle: |det| near EPSILON, where the
    reference's f32 barycentrics are least accurate."""
    A, B, C, N = _verts(tris)
    pos, _ = _bounce_like_rays(tris, n, rng)
    j = rng.integers(0, len(tris), n)
    w = rng.dirichlet([1, 1, 1], n)
    target = w[:, :1] * A[j] + w[:, 1:2] * B[j] + w[:, 2:] * C[j]
    d = _unit(target - pos)
    d = d - np.sum(d * N[j], 1, keepdims=True) * N[j]  # into the target's plane
    d = _unit(d + 1e-30) - N[j] * (10.0 ** rng.uniform(-6, -1, (n, 1)))
    return pos, d


def _self_rays(tris, n, rng):
    """Origins on (or a hair off) a triangle's plane, aimed along that plane and slightly through it: the
    reference's dot(AC, (pos - A) x AB) near 0, where the first-bounce reach mask decides."""
    A, B, C, N = _verts(tris)
    k = rng.integers(0, len(tris), n)
    w = rng.dirichlet([1, 1, 1], n) * 1.4 - 0.2  # inside and just outside the triangle
    pos = w[:, :1] * A[k] + w[:, 1:2] * B[k] + w[:, 2:] * C[k]
    pos += N[k] * (rng.normal(size=(n, 1)) * 10.0 ** rng.uniform(-8, -3, (n, 1)))
    w2 = rng.dirichlet([1, 1, 1], n)
    d = _unit(w2[:, :1] * A[k] + w2[:, 1:2] * B[k] + w2[:, 2:] * C[k] - pos + 1e-30)
    d = d - N[k] * np.sum(d * N[k], 1, keepdims=True)
    return pos, _unit(d + 1e-30) - N[k] * (rng.choice([-1.0, 1.0], (n, 1)) * 10.0 ** rng.uniform(-7, 0, (n, 1)))


def _free_rays(tris, n, rng):
    A, B, C, _ = _verts(tris)
    lo = np.minimum(np.minimum(A, B), C).min(0)
    hi = np.maximum(np.maximum(A, B), C).max(0)
    ext = hi - lo
    pos = lo - 0.5 * ext + rng.random((n, 3)) * 2 * ext
    return pos, _unit(rng.normal(size=(n, 3)))


def _rays(tris, n, rng):
    gens = (_bounce_like_rays, _aimed_rays, _grazing_rays, _self_rays, _free_rays)
    parts = [g(tris, n, rng) for g in gens]
    r = np.zeros(len(gens) * n, RAY_DT)
    pos = np.concatenate([p for p, _ in parts]).astype(np.float32)
    d = np.concatenate([d for _, d in parts]).astype(np.float32)
    for i, c in enumerate("xyz"):
        r["pos"][c] = pos[:, i]
        r["dir"][c] = d[:, i]
    return r


def _scaled(tris, s):
    t = tris.copy()
    for v in ("posA", "posB", "posC"):
        for c in "xyz":
            t[v][c] = (t[v][c].astype(np.float64) * s).astype(np.float32)
    return t


@pytest.mark.parametrize("name,scale", [("ultracomplex", 1.0), ("complex", 1.0), ("cube", 1.0),
                                        ("ultracomplex", 40.0), ("ultracomplex", 0.02), ("fsuzane", 1.0),
                                        ("4geoms", 1.0), ("default", 1.0), ("suzannes", 1.0), ("suzannes", 25.0)])
def test_cluster_culling_is_sound(name, scale, gpu_available):
    """suzannes.obj (5,208 triangles, 21 chunks) also checks the chunk balls of rtc_render_chain's first level."""
    tris, _ = load_tris(name)
    tris = _scaled(tris, scale)
    rng = np.random.default_rng(1234 + int(scale * 100))
    rays = _rays(tris, 250_000 if len(tris) <= 256 else 40_000, rng)
    r = rt.cluster_bound_probe(tris, rays)
    print(name, scale, r)
    assert r["violations"] == 0, r
    assert r["reach_violations"] == 0, r
    assert r["hits"] > 1_000
    if scale <= 1.0:  # aligned_normal's margin is absolute (EPSILON): large triangles are never "aligned"
        assert r["unreachable"] > 0
    if len(tris) > 16 and scale == 1.0:
        assert r["culled"] > r["tests"] // 8  # the bound is not vacuous

"""Write a Triangle[] back out as OBJ + MTL such that the reference's loader reproduces it byte for byte.

The reference binary (oracle/_ref/rtc_ref, the reference's own main) reads scenes only from OBJ files, and the
GPU box has no /root/reference; bench.py and the CLI tests therefore export the committed Triangle[] fixtures
(tests/golden/scenes/*.tris) to a temporary OBJ.  Inverse of loadOBJTriangles (raytracing.c:100-147: x and y
of positions and normals negated) and loadObj / loadMtl (objloader.c:221-551: the face normal is the `vn` of
the first face vertex; Kd -> color; the first Ke component -> emission; Ns -> smoothness = (float)sqrt(0.001 *
Ns), objloader.c:272).  Not part of the product.
"""
from __future__ import annotations

import numpy as np


def _ns_for(smoothness: np.float32) -> np.float32:
    """A float Ns with (float)sqrt(0.001 * (double)Ns) == smoothness (objloader.c:272)."""
    s = np.float32(smoothness)
    guess = np.float32(np.float64(s) * np.float64(s) / 0.001)
    cand = guess
    for _ in range(64):
        got = np.float32(np.sqrt(0.001 * np.float64(cand)))
        if got == s:
            return cand
        cand = np.nextafter(cand, np.float32(np.inf) if got < s else np.float32(-np.inf))
    raise ValueError(f"no Ns reproduces smoothness {float(s)!r}")


def write_obj(path: str, tris: np.ndarray) -> None:
    """OBJ (+ `<path>.mtl` when any triangle has a non-default material) whose loadOBJTriangles result is
    `tris` byte for byte (x, y negated back; one `vn` per face; one material per distinct (color, emission,
    smoothness))."""
    mats: dict = {}
    face_mat = []
    for t in tris:
        m = t["mat"]
        key = (np.float32(m["color"]["x"]).tobytes(), np.float32(m["color"]["y"]).tobytes(),
               np.float32(m["color"]["z"]).tobytes(), np.float32(m["emissionStrength"]).tobytes(),
               np.float32(m["smoothness"]).tobytes())
        if key not in mats:
            mats[key] = (len(mats), m)
        face_mat.append(mats[key][0])
    default = all(np.frombuffer(b"".join(k), np.float32).tolist() == [1.0, 1.0, 1.0, 0.0, 0.0] for k in mats)
    mtl = path + ".mtl"
    with open(path, "w") as f:
        if mats and not default:
            f.write(f"mtllib {mtl.rsplit('/', 1)[-1]}\n")
        for t in tris:
            for v in ("posA", "posB", "posC"):
                f.write(f"v {-t[v]['x']:.9g} {-t[v]['y']:.9g} {t[v]['z']:.9g}\n")
            f.write(f"vn {-t['normal']['x']:.9g} {-t['normal']['y']:.9g} {t['normal']['z']:.9g}\n")
        cur = -1
        for i in range(len(tris)):
            if not default and face_mat[i] != cur:
                cur = face_mat[i]
                f.write(f"usemtl m{cur}\n")
            f.write(f"f {3 * i + 1}/1/{i + 1} {3 * i + 2}/1/{i + 1} {3 * i + 3}/1/{i + 1}\n")
    if mats and not default:
        with open(mtl, "w") as f:
            for _, (k, m) in sorted((v[0], v) for v in mats.values()):
                f.write(f"newmtl m{k}\n")
                f.write(f"Ns {float(_ns_for(m['smoothness'])):.9g}\n")
                f.write(f"Kd {float(m['color']['x']):.9g} {float(m['color']['y']):.9g} {float(m['color']['z']):.9g}\n")
                f.write(f"Ke {float(m['emissionStrength']):.9g} 0 0\n\n")

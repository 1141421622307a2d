"""Generate tests/golden/function_goldens.npz: per-function golden vectors of the CPU oracle
(SURVEY.md 8c "per-function vectors for hit/scatter/pdf/texture"), so that a divergence in one
hot-path function can be localised (closest hits are in oracle_goldens.npz).

    python tests/golden/make_function_goldens.py      (needs oracle/build/liboracle.so, librtamd.so)

For each scene below, seeded inputs are evaluated by oracle_probe (oracle/oracle.c; record i draws
from its own tier-B Philox stream: key = SEED, pid = i, sample 0) for
  scatter       every material kind the scene has (Lambertian with its light mixture, Metal, Dielectric,
                DiffuseLight -> emitted, Isotropic), random rays / hit records   (src/Lib.hs:822-885)
  htbl_random   origins inside the scene, on the lights tree                     (src/Lib.hs:707-724)
  htbl_pdf      origins and directions, half of them towards the lights          (src/Lib.hs:673-705)
  texture       every texture of the scene (constant, checker, Perlin, image)    (src/Lib.hs:496-513)
  get_ray       s, t in [0, 1] with the scene's camera (thin lens, time draw)   (src/Lib.hs:1253-1267)
Keys: <scene>_<fn>_in, <scene>_<fn>_out. Self-generated (no GHC exists to produce reference ones).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402
import rtamd  # noqa: E402

OUT = os.path.join(HERE, "function_goldens.npz")
SEED = 77
# scene -> (camera, scale of positions (lo, hi), earth?)
SCENES = {
    "cornell": ("cornell", (0.0, 555.0), False),
    "cornell_smoke": ("cornell", (0.0, 555.0), False),
    "random_book_one": ("random_scene", (-12.0, 12.0), False),
    "next_week_final": ("next_week", (-50.0, 600.0), True),
    "random": ("random_scene", (-12.0, 12.0), True),
    "two_perlin_spheres": ("two_spheres", (-5.0, 5.0), False),
    "simple_light": ("two_spheres", (-5.0, 5.0), False),
}


def earth():
    return np.load(os.path.join(HERE, "earthmap_rgb8.npz"))["rgb"]


def make_scene(name):
    cam, scale, use_earth = SCENES[name]
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024), earth=earth() if use_earth else None)
    return sc, rtamd.camera(cam, 64, 48), scale


def unit(v):
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def inputs(name, sc, scale, rng):
    lo, hi = scale
    mats = sc.materials
    out = {}
    # scatter: up to 8 materials of each kind, 48 records each
    pick = []
    for kind in range(5):
        ids = np.flatnonzero(mats["type"] == kind)
        pick += list(ids[:8])
    recs = []
    for m in pick:
        n = 48
        o = rng.uniform(lo, hi, (n, 3))
        d = rng.normal(0, 1, (n, 3)) * rng.uniform(0.2, 3.0, (n, 1))
        tm = rng.uniform(0, 1, (n, 1))
        t = rng.uniform(0.01, 10.0, (n, 1))
        p = rng.uniform(lo, hi, (n, 3))
        nn = unit(rng.normal(0, 1, (n, 3)))
        nn[: n // 8] = np.eye(3)[rng.integers(0, 3, n // 8)] * rng.choice([-1.0, 1.0], (n // 8, 1))  # axis normals
        uv = rng.uniform(0, 1, (n, 2))
        ff = rng.integers(0, 2, (n, 1)).astype(np.float64)
        recs.append(np.concatenate([o, d, tm, t, p, nn, uv, ff, np.full((n, 1), float(m))], axis=1))
    out["scatter"] = np.concatenate(recs)
    if sc.desc.lights_root >= 0:
        n = 384
        org = rng.uniform(lo + 0.1 * (hi - lo), hi - 0.1 * (hi - lo), (n, 3))
        out["htbl_random"] = org
        dirs = pyoracle.probe(sc, "htbl_random", org, seed=SEED)[:, :3]
        v = rng.normal(0, 1, (n, 3))
        v[: n // 2] = dirs[: n // 2]  # towards the lights: non-zero pdfs
        out["htbl_pdf"] = np.concatenate([org, v], axis=1)
    recs = []
    kinds = sc.textures["type"]
    tids = list(np.flatnonzero(kinds != 0)) + list(np.flatnonzero(kinds == 0)[:8])  # every non-constant one
    for tid in sorted(tids):
        n = 64
        uv = rng.uniform(0, 1, (n, 2))
        uv[:4] = [[0, 0], [1, 1], [0, 1], [1, 0]]  # image texture clamps at the edges
        p = rng.uniform(lo, hi, (n, 3))
        recs.append(np.concatenate([np.full((n, 1), float(tid)), uv, p], axis=1))
    out["texture"] = np.concatenate(recs)
    out["get_ray"] = rng.uniform(0, 1, (256, 2))
    return out


def build():
    g = {}
    rng = np.random.default_rng(2024)
    for name in SCENES:
        sc, cam, scale = make_scene(name)
        for fn, x in inputs(name, sc, scale, rng).items():
            g[f"{name}_{fn}_in"] = x
            g[f"{name}_{fn}_out"] = pyoracle.probe(sc, fn, x, seed=SEED, cam=cam)
    return g


if __name__ == "__main__":
    g = build()
    np.savez_compressed(OUT, **g)
    print(OUT, os.path.getsize(OUT), "bytes;", len(g) // 2, "vectors")

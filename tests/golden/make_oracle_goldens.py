"""Generate tests/golden/oracle_goldens.npz: golden vectors of the CPU oracle (oracle/oracle.c).

These are SELF-GENERATED fixtures (SURVEY.md 8c "build-generated goldens"): the reference has no
tests and its Haskell toolchain is absent, so they pin the oracle and the HIP path against
regressions and against each other, not against a GHC run. The reference-produced pin is
statistical (cornell1000_blocks.npz, tests/test_oracle.py).

    python tests/golden/make_oracle_goldens.py      (needs oracle/build/liboracle.so and librtamd.so)

Contents (key: what it holds):
  rng_*        randGen 1024: the first 32 nextWord64 words and randomDouble draws (src/Random.hs)
  c1b_*        config 1 (three_spheres, randomSceneCamera, 200x100, 10 spp, depth 10), tier B seed
               1024: RGB8 image, and the linear (pre-albedoToColor) averages of rows 0..7
  c1a_*        the same in tier A (app/Main.hs:47-49 generators, deterministic harness of
               rtamd.column_gens): RGB8, linear rows 0..7, the end-of-stream generators
  cba_*        makeCornellBoxScene, cornellCamera, 64x64, 16 spp, depth 50, tier A
  hits_<scene> closest hits (rt_debug_closest_hits layout) of 512 seeded rays, and the rays
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

OUT = os.path.join(HERE, "oracle_goldens.npz")
LIN_ROWS = 8


def hit_rays(name, n=512, seed=23):
    rng = np.random.default_rng(seed)
    if name in ("random_book_one", "three_spheres"):
        o = np.array([13.0, 2.0, 3.0]) + rng.normal(0, 0.5, (n, 3))
        d = np.array([-13.0, -2.0, -3.0]) + rng.normal(0, 3.0, (n, 3))
    else:
        o = rng.uniform(20, 530, (n, 3))
        d = rng.normal(0, 1, (n, 3))
    return np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)


def build():
    g = {}
    words, _ = pyoracle.words(rtamd.randGen(1024), 32)
    g["rng_words"] = np.array(words, dtype=np.uint64)
    draws, _ = pyoracle.draws(rtamd.randGen(1024), 32)
    g["rng_draws"] = np.array(draws)

    sc, g1 = rtamd.make_scene("three_spheres", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 200, 100)
    rgb, lin, _, _ = pyoracle.render(sc, cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_PHILOX, seed=1024))
    g["c1b_rgb"], g["c1b_lin"] = rgb, lin[:LIN_ROWS]
    gens = rtamd.column_gens(g1, 200)
    rgb, lin, go, _ = pyoracle.render(sc, cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_EXACT), col_gens=gens)
    g["c1a_rgb"], g["c1a_lin"], g["c1a_gens_in"], g["c1a_gens_out"] = rgb, lin[:LIN_ROWS], gens, go

    sc, g1 = rtamd.make_scene("cornell", rtamd.randGen(1024))
    cam = rtamd.camera("cornell", 64, 64)
    gens = rtamd.column_gens(g1, 64)
    rgb, lin, go, _ = pyoracle.render(sc, cam, rtamd.make_params(64, 64, 16, 50, rtamd.RT_RNG_EXACT), col_gens=gens)
    g["cba_rgb"], g["cba_lin"], g["cba_gens_in"], g["cba_gens_out"] = rgb, lin, gens, go

    for name in ("random_book_one", "cornell"):
        sc, _ = rtamd.make_scene(name, rtamd.randGen(1024))
        rays = hit_rays(name)
        g[f"hits_{name}_rays"] = rays
        g[f"hits_{name}"] = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    return g


if __name__ == "__main__":
    g = build()
    np.savez_compressed(OUT, **g)
    print(OUT, os.path.getsize(OUT), "bytes;", ", ".join(f"{k}{tuple(v.shape)}" for k, v in g.items()))

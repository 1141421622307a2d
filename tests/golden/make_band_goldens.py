"""Generate tests/golden/bench_bands.npz: oracle renders of full-width row bands of the EXACT bench
frames (bench.py CONFIGS), so that the GPU test can render each whole frame through
the path bench.py times (rt_render_shard_async + rt_assemble_async, the same kernel instantiation,
chunking and work decomposition) and compare the band.

The frame geometry fixes the tier-B definition (rt_sample_chunk depends on W*H and spp), so each band
is rendered by the oracle with the full frame's parameters and only its rows evaluated
(oracle_render_rows). Self-generated fixtures: the reference has no tests and no GHC
exists here; they pin the HIP path against the oracle at the bench launches.

    python tests/golden/make_band_goldens.py          (needs oracle/build/liboracle.so, librtamd.so)

Bands (key prefix: frame, rows):
  c2_  makeRandomSceneBookOne 1200x800, 500 spp, depth 50 (8-sample chunks x 63), rows 396..403
  c3_  makeCornellBoxScene 600x600, 1000 spp, depth 50 (8-sample chunks x 125), rows 296..303
  c4_  makeNextWeekFinalScene + earth raster 800x800, 1000 spp, depth 50 (8-sample chunks), rows 396..403
  c5_  stress 100k spheres 3840x2160 at 4 spp, depth 50 (the global-memory 4-wide kernel), rows 1079..1080
  c5b_ the C5 frame at its bench spp, 2000 (16-sample chunks x 125, rendered in chunk batches), row 1080
  c4s_ the C4 frame at 16 spp (two chunks per pixel), rows 398..401
  c2z_, c4z_, c5z_, c5bz_  the C2 / C4 / C5 bands again with RT_FLAG_NAN_ZERO (include/rt.h, a parity
       diagnostic): the reference's Lambertian light-mixture quirk makes 99.9 % of
       the C2 band's channels and all of C4's NaN at the bench spp, so the plain bands compare little
       more than NaN masks; with the flag each sample's finite colour reaches the average, so the same
       launches are compared sample by sample
Each band stores rgb (uint8), lin (float64, the pre-albedoToColor averages) and the frame
parameters (w, h, spp, depth, seed, r0, flags).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402
import rtamd  # noqa: E402

OUT = os.path.join(HERE, "bench_bands.npz")

Z = rtamd.RT_FLAG_NAN_ZERO
# (key, scene, camera, W, H, spp, depth, param, earth, r0, rows, flags)
BANDS = [
    ("c2", "random_book_one", "random_scene", 1200, 800, 500, 50, 0, False, 396, 8, 0),
    ("c3", "cornell", "cornell", 600, 600, 1000, 50, 0, False, 296, 8, 0),
    ("c4", "next_week_final", "next_week", 800, 800, 1000, 50, 0, True, 396, 8, 0),
    ("c5", "stress_spheres", "random_scene", 3840, 2160, 4, 50, 100000, False, 1079, 2, 0),
    ("c5b", "stress_spheres", "random_scene", 3840, 2160, 2000, 50, 100000, False, 1080, 1, 0),
    ("c4s", "next_week_final", "next_week", 800, 800, 16, 50, 0, True, 398, 4, 0),
    ("c2z", "random_book_one", "random_scene", 1200, 800, 500, 50, 0, False, 396, 8, Z),
    ("c4z", "next_week_final", "next_week", 800, 800, 1000, 50, 0, True, 396, 8, Z),
    ("c5z", "stress_spheres", "random_scene", 3840, 2160, 4, 50, 100000, False, 1079, 2, Z),
    ("c5bz", "stress_spheres", "random_scene", 3840, 2160, 2000, 50, 100000, False, 1080, 1, Z),
]
SEED = 1024


def earth():
    return np.load(os.path.join(HERE, "earthmap_rgb8.npz"))["rgb"]


def band(key, scene, camname, W, H, spp, depth, param, use_earth, r0, rows, flags, nthreads=0):
    sc, _ = rtamd.make_scene(scene, rtamd.randGen(1024), param=param, earth=earth() if use_earth else None)
    cam = rtamd.camera(camname, W, H)
    p = rtamd.make_params(W, H, spp, depth, rtamd.RT_RNG_PHILOX, seed=SEED, flags=flags)
    rgb, lin, _, _ = pyoracle.render(sc, cam, p, rows=(r0, r0 + rows), nthreads=nthreads)
    return rgb, lin


def build(keys=None):
    g = {}
    for key, scene, camname, W, H, spp, depth, param, use_earth, r0, rows, flags in BANDS:
        if keys and key not in keys:
            continue
        t0 = time.time()
        rgb, lin = band(key, scene, camname, W, H, spp, depth, param, use_earth, r0, rows, flags)
        g[f"{key}_rgb"], g[f"{key}_lin"] = rgb, lin
        g[f"{key}_frame"] = np.array([W, H, spp, depth, SEED, r0, flags], dtype=np.int64)
        print(f"{key}: {W}x{H}x{spp} rows {r0}..{r0 + rows - 1}: {time.time() - t0:.1f} s, "
              f"NaN channels {np.isnan(lin).mean():.3f}", flush=True)
    return g


if __name__ == "__main__":
    keys = sys.argv[1:]
    g = build(keys)
    if keys and os.path.exists(OUT):  # (rebuild some bands, keep the others)
        old = dict(np.load(OUT))
        old.update(g)
        g = old
    np.savez_compressed(OUT, **g)
    print(OUT, os.path.getsize(OUT), "bytes")

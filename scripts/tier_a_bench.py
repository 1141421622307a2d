"""Tier A (RT_RNG_EXACT: the reference's per-column SplitMix stream, one lane per image column, the caller's
tree) timed on the GPU beside the oracle's tier-A render of the same frame on the host's cores — the
drop-in path's speed, which bench.py does not measure (its metric is tier B). Prints one JSON line per
case. usage: python scripts/tier_a_bench.py [--threads 16]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
import rtamd  # noqa: E402

CASES = [  # (scene, camera, W, H, spp, depth)
    ("three_spheres", "random_scene", 200, 100, 10, 10),   # C1, the reference's CPU-runnable case
    ("cornell", "cornell", 200, 200, 16, 50),
    ("random_book_one", "random_scene", 300, 200, 8, 50),
]

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
a = ap.parse_args()
ctx = rtamd.Context(0)
for name, camname, W, H, spp, depth in CASES:
    sc, g1 = rtamd.make_scene(name, rtamd.randGen(1024))
    cam = rtamd.camera(camname, W, H)
    p = rtamd.make_params(W, H, spp, depth, rtamd.RT_RNG_EXACT, seed=1024)
    gens = rtamd.column_gens(g1, W)
    ctx.upload(sc)
    ctx.render(cam, p, gens)  # warm-up
    t0 = time.perf_counter()
    rgb, _, _ = ctx.render(cam, p, gens)
    gpu_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    rgb_o, _, _, _ = pyoracle.render(sc, cam, p, col_gens=gens, nthreads=a.threads, linear=False)
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"scene": name, "size": [W, H, spp, depth], "tier": "A", "gpu_s": round(gpu_s, 4),
                      "gpu_msamples_s": round(W * H * spp / gpu_s / 1e6, 3), "cpu_s": round(cpu_s, 3),
                      "cpu_threads": a.threads, "bytes_equal": float(np.mean(rgb == rgb_o))}), flush=True)
ctx.close()

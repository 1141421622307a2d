"""Render a bench config (tier B) and print the SHA-256 of its RGB8 bytes and fp64 linear averages: the
A/B check that a variant build renders the same image as the tree (scripts/ab.py builds _var_* dirs that
carry this script). usage: python scripts/img_hash.py [--config c2] [--spp 16]"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ray-tracing_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--spp", type=int, default=16)
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"] if cfg.get("earth") else None
scene, _ = rtamd.make_scene(cfg["scene"], rtamd.randGen(1024), param=cfg.get("param", 0), earth=earth)
cam = rtamd.camera(cfg["camera"], cfg["W"], cfg["H"])
ctx = rtamd.Context(0)
ctx.upload(scene)
p = rtamd.make_params(cfg["W"], cfg["H"], a.spp, cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024)
rgb, lin, _ = ctx.render(cam, p, linear=True)
print(f"{a.config} at {a.spp} spp: rgb {hashlib.sha256(np.ascontiguousarray(rgb).tobytes()).hexdigest()[:16]} "
      f"lin {hashlib.sha256(np.ascontiguousarray(lin).tobytes()).hexdigest()[:16]}")
ctx.close()

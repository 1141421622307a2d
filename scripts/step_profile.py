"""Where a binary / mixed walk's steps spend their time (rt_render_step_profile, counting build): wave
time and count of the walk's steps by the set of node kinds their lanes were at, plus the loop's phase
split. usage: python scripts/step_profile.py [--config c4] [--spp 32]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ray-tracing_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--spp", type=int, default=32)
ap.add_argument("--json", default="")
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"] if cfg.get("earth") else None
scene, _ = rtamd.make_scene(cfg["scene"], rtamd.randGen(1024), param=cfg.get("param", 0), earth=earth)
cam = rtamd.camera(cfg["camera"], cfg["W"], cfg["H"])
ctx = rtamd.Context(0)
ctx.upload(scene)
p = rtamd.make_params(cfg["W"], cfg["H"], a.spp, cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024)
prof = ctx.step_profile(cam, p)
work = ctx.render_work(cam, p)
tot = sum(v[0] for v in prof.values())
steps = sum(v[1] for v in prof.values())
print(f"{a.config} at {a.spp} spp: {steps} wave steps, {tot / max(1, steps):.0f} ticks per step; phase split "
      f"{ {k: round(v, 3) for k, v in work['phase_split'].items()} }")
print(f"{'kinds':28s} {'time':>7s} {'steps':>7s} {'ticks/step':>10s}")
for k, (ticks, n) in sorted(prof.items(), key=lambda x: -x[1][0]):
    print(f"{k:28s} {ticks / tot:7.3f} {n / steps:7.3f} {ticks / n:10.0f}")
per_kind = {}
for k, (ticks, n) in prof.items():
    for kind in k.split("+"):
        per_kind.setdefault(kind, [0, 0])
        per_kind[kind][0] += ticks
        per_kind[kind][1] += n
print("steps containing each kind:", {k: (round(v[0] / tot, 3), round(v[1] / steps, 3)) for k, v in per_kind.items()})
if a.json:
    with open(a.json, "w") as f:
        json.dump({"config": a.config, "spp": a.spp, "profile": prof, "work": work}, f)
ctx.close()

"""Where C4's time goes by object group: next_week_final's parts (tests/nwf_parts.py) rendered at the C4
camera and size, all of them and all but one group at a time, tier B, timed with rt_frame_timing (kernel
ms) plus the counting build's work per sample. usage: python scripts/c4_parts.py [--spp 32]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "tests")]
import nwf_parts  # noqa: E402
import rtamd  # noqa: E402

ALL = ["boxes", "light", "moving", "glass", "metal", "fog1", "fog2", "perlin", "inst"]
ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=32)
a = ap.parse_args()
ctx = rtamd.Context(0)
cam = rtamd.camera("next_week", 800, 800)
p = rtamd.make_params(800, 800, a.spp, 50, rtamd.RT_RNG_PHILOX, seed=1024)
cases = [("all", ALL)] + [("-" + g, [x for x in ALL if x != g]) for g in ALL] + [
    ("boxes", ["boxes"]), ("inst", ["inst"]), ("boxes+fog2", ["boxes", "fog2"]),
    ("inst_flat", [x for x in ALL if x != "inst"] + ["inst_flat"])]
for name, parts in cases:
    sc, _ = nwf_parts.scene(parts)
    ctx.upload(sc)
    ctx.render(cam, p)  # warm-up
    ms = []
    for _ in range(2):
        ctx.render(cam, p)
        ms.append(ctx.frame_timing()["kernel_ms"][0])
    w = ctx.render_work(cam, p)
    n = max(1, w["samples"])
    per = {k: round(w[k] / n, 2) for k in ("segments", "box_tests", "wide_nodes", "prim_tests", "other_tests")}
    print(f"{name:12s} {min(ms):8.1f} ms  {per}", flush=True)
ctx.close()

"""A small tier-B render of next_week_final (media in the 4-wide world tree) against the oracle: the first
thing to run after a change to the media walk (exits non-zero on any error)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle  # noqa: E402
import rtamd  # noqa: E402
from conftest import parity  # noqa: E402

earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"]
ctx = rtamd.Context(0)
for name, cam in (("next_week_final", "next_week"), ("cornell_smoke", "cornell")):
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024), earth=earth if name == "next_week_final" else None)
    ctx.upload(sc)
    c = rtamd.camera(cam, 64, 64)
    for flags in (rtamd.RT_FLAG_NAN_ZERO, 0):
        p = rtamd.make_params(64, 64, 8, 50, rtamd.RT_RNG_PHILOX, seed=7, flags=flags)
        rgb, lin, _ = ctx.render(c, p, linear=True)
        rgb_o, lin_o, _, _ = pyoracle.render(sc, c, p)
        ok, eq, dmax = parity(lin, lin_o, rgb, rgb_o)
        print(f"{name} flags {flags}: {ctx.last_launch()['loop']=} channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, "
              f"max |d| {dmax:.3g}", flush=True)
ctx.close()

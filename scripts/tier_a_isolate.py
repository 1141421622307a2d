"""Tier-A (RT_RNG_EXACT) GPU-vs-oracle on pieces of next_week_final (Scenes.hs:414-466), one feature group
per scene, with RT_FLAG_SHARED_LIBM on both sides (so only the path logic can differ): which part makes
the columns' streams diverge. Prints, per scene, equal bytes and the columns whose end generators differ.

    python scripts/tier_a_isolate.py [W H spp]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle")]
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle  # noqa: E402
import rtamd  # noqa: E402
from nwf_parts import scene  # noqa: E402


def main():
    W, H, spp = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 32, 3)
    ctx = rtamd.Context(0)
    cases = [["boxes", "light"], ["moving", "glass", "metal", "light"], ["fog1", "light", "glass"],
             ["fog2", "boxes", "light"], ["inst", "light"], ["perlin", "light"]]
    earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"]
    full, g1 = rtamd.make_scene("next_week_final", rtamd.randGen(1024), earth=earth)
    cam = rtamd.camera("next_week", W, H)
    for parts in cases + [None]:
        sc, g = (full, g1) if parts is None else scene(parts)
        gens = rtamd.column_gens(g, W)
        ctx.upload(sc)
        for cull in (0, rtamd.RT_FLAG_REFERENCE_CULL):
            p = rtamd.make_params(W, H, spp, 50, rtamd.RT_RNG_EXACT, flags=rtamd.RT_FLAG_SHARED_LIBM | cull)
            rgb_g, _, gg = ctx.render(cam, p, gens, want_gens=True)
            rgb_o, _, go, _ = pyoracle.render(sc, cam, p, col_gens=gens)
            bad = np.nonzero(~(gg == go).all(axis=1))[0]
            print(f"{'+'.join(parts) if parts else 'next_week_final':28s} {'ref-cull' if cull else 'joint   '} bytes "
                  f"equal {float((rgb_g == rgb_o).mean()):.4f}, columns diverged {len(bad)}/{W} {bad[:8].tolist()}",
                  flush=True)
            if len(bad) and not cull:
                first_divergence(ctx, sc, cam, p, gens, int(bad[0]))
    ctx.close()



def first_divergence(ctx, sc, cam, p, gens, col):
    """Trace column `col` on both sides; print the first differing segment record and its neighbours."""
    a = ctx.exact_trace(cam, p, gens, col)
    b = pyoracle.exact_trace(sc, cam, p, gens, col)
    n = min(len(a), len(b))
    same = np.all((a[:n] == b[:n]) | (np.isnan(a[:n]) & np.isnan(b[:n])), axis=1)
    bad = np.nonzero(~same)[0]
    print(f"column {col}: {len(a)} device / {len(b)} oracle segments; first difference at record "
          f"{bad[0] if len(bad) else None}")
    if len(bad):
        k = bad[0]
        np.set_printoptions(precision=17, linewidth=200)
        for i in range(max(0, k - 2), min(n, k + 2)):
            print("  dev", i, a[i, :9].tolist(), hex(a[i, 9:10].view(np.uint64)[0]))
            print("  ora", i, b[i, :9].tolist(), hex(b[i, 9:10].view(np.uint64)[0]))
    return a, b


if __name__ == "__main__":
    main()

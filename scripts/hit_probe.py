"""Closest hits on axis-aligned rays grazing the box field (the Lambertian quirk's +x light direction
from points on box tops): GPU walks against the oracle. Prints the mismatching rays.

    python scripts/hit_probe.py [scene parts, default fog2+boxes+light]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle  # noqa: E402
import rtamd  # noqa: E402
from nwf_parts import grazing_rays as rays_for, scene  # noqa: E402


def main():
    parts = (sys.argv[1] if len(sys.argv) > 1 else "fog2+boxes+light").split("+")
    sc, _ = scene(parts)
    ctx = rtamd.Context(0)
    ctx.upload(sc)
    rays = rays_for(sc, 1 << 16, np.random.default_rng(3))
    ref = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    for name, flags in (("recursive joint", 0), ("recursive ref-cull", rtamd.RT_FLAG_REFERENCE_CULL),
                        ("resumable joint", rtamd.RT_DEBUG_RESUMABLE)):
        try:
            got = ctx.closest_hits(rays, 1e-4, np.inf, seed=3, flags=flags)
        except rtamd.RTError as e:
            print(name, e)
            continue
        same = np.all((got == ref) | (np.isnan(got) & np.isnan(ref)), axis=1)
        # medium hits (Isotropic phase material, normal (1, 0, 0)): t through OCML vs glibc log, ulps apart
        mats = sc.materials["type"]
        med = (ref[:, 0] == 1) & (got[:, 0] == 1) & (mats[ref[:, 11].astype(int)] == 4) & (ref[:, 11] == got[:, 11])
        close = med & (np.abs(got[:, 1] - ref[:, 1]) <= 8 * np.spacing(np.abs(ref[:, 1])))
        real = ~same & ~close
        print(f"{name}: {int((~same).sum())} of {len(rays)} rays differ, {int((~same & close).sum())} of them medium t "
              f"within 8 ulps; hits {int(ref[:, 0].sum())}", flush=True)
        for i in np.nonzero(real)[0][:6]:
            print("  ray", rays[i].tolist())
            print("  gpu", got[i].tolist())
            print("  ora", ref[i].tolist())
    ctx.close()


if __name__ == "__main__":
    main()

"""Pieces of next_week_final (src/Scenes.hs:414-466) as separate worlds, built through the constructor
API (rtamd.Builder): the box field, the light, the moving / glass / metal spheres, the two media, the
Perlin sphere and the 1000-sphere instance. Used by the tier-A and grazing-ray parity tests and by
scripts/tier_a_isolate.py / scripts/hit_probe.py to localise a divergence to one feature."""
import numpy as np

import rtamd


def scene(parts):
    b = rtamd.Builder(rtamd.randGen(1024))
    items = []
    lam = lambda r, g, bl: b.lambertian(b.constantColor(r, g, bl))  # noqa: E731
    if "boxes" in parts:
        ground = lam(0.48, 0.83, 0.53)
        rng = np.random.default_rng(0)
        bx = []
        for i in range(20):
            for j in range(20):
                x0, z0 = i * 100.0 - 1000, j * 100.0 - 1000
                bx.append(b.cuboid((x0, 0.0, z0), (x0 + 100, float(rng.uniform(1, 101)), z0 + 100), ground))
        items.append(b.makeBVH((0.0, 1.0), bx))
    if "light" in parts:
        items.append(b.rect(rtamd.XZPlane, 113, 443, 127, 432, 554, b.diffuseLight(b.constantColor(7, 7, 7))))
    if "moving" in parts:
        items.append(b.movingSphere((400, 400, 200), (430, 400, 200), 0.0, 1.0, 50, lam(0.7, 0.3, 0.1)))
    if "glass" in parts:
        items.append(b.sphere((260, 150, 45), 50, b.dielectric(1.5)))
    if "metal" in parts:
        items.append(b.sphere((0, 150, 145), 50, b.metal(b.constantColor(0.8, 0.8, 0.9), 10.0)))
    if "fog1" in parts:
        bd = b.sphere((360, 150, 145), 70, b.dielectric(1.5))
        items += [bd, b.constantMedium(0.2, b.constantColor(0.2, 0.4, 0.9), bd)]
    if "fog2" in parts:
        bd = b.sphere((0, 0, 0), 5000, b.dielectric(1.5))
        items.append(b.constantMedium(0.0001, b.constantColor(1, 1, 1), bd))
    if "perlin" in parts:
        items.append(b.sphere((220, 280, 300), 80, b.lambertian(b.makePerlin(0.1))))
    if "inst" in parts or "inst_flat" in parts:
        white = lam(0.73, 0.73, 0.73)
        rng = np.random.default_rng(1)
        cs = rng.uniform(0, 165, (1000, 3))
        if "inst" in parts:
            sp = [b.sphere(tuple(c), 10, white) for c in cs]
            items.append(b.translate((-100, 270, 395), b.rotate(rtamd.YAxis, 15, b.makeBVH((0.0, 1.0), sp))))
        else:  # (perf experiments only: the same spheres placed in world space, no instance frame)
            a = np.radians(15.0)
            w = np.stack([np.cos(a) * cs[:, 0] + np.sin(a) * cs[:, 2], cs[:, 1],
                          -np.sin(a) * cs[:, 0] + np.cos(a) * cs[:, 2]], axis=1) + np.array([-100, 270, 395])
            items.append(b.makeBVH((0.0, 1.0), [b.sphere(tuple(c), 10, white) for c in w]))
    world = b.makeBVH((0.0, 1.0), items) if len(items) > 1 else items[0]
    return b.finish(world, -1, (0.0, 0.0, 0.0)), b.gen


def grazing_rays(sc, n, rng):
    """Rays like the Lambertian quirk's +x light direction from a box top (Lib.hs:829-835 with lights
    Unhittable): origins on (or one ulp off) a cuboid's top face, axis-aligned directions along x or z.
    Such a ray lies in a face plane of the boxes around it: exact ties between neighbouring faces, rect
    hits at t = NaN (the plane it runs in), and boxes the reference's per-axis test rejects for a NaN
    slab quotient."""
    nodes = sc.nodes
    cub = nodes[nodes["type"] == rtamd.RT_NODE_CUBOID]
    k = rng.integers(0, len(cub), n)
    lo, hi = cub["f"][k, :3], cub["f"][k, 3:]
    o = lo + (hi - lo) * rng.random((n, 3))
    o[:, 1] = hi[:, 1]
    m = rng.random(n)
    o[m < 0.25, 1] = np.nextafter(hi[m < 0.25, 1], -np.inf)
    o[(m >= 0.25) & (m < 0.5), 1] = np.nextafter(hi[(m >= 0.25) & (m < 0.5), 1], np.inf)
    d = np.zeros((n, 3))
    ax = rng.integers(0, 4, n)
    d[ax == 0, 0] = 1.0
    d[ax == 1, 0] = -1.0
    d[ax == 2, 2] = 1.0
    d[ax == 3, 2] = -1.0
    return np.concatenate([o, d, rng.random((n, 1))], axis=1)

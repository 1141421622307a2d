"""The BVH box test one record at a time (RT_PROBE_BOX; rt_trace.h box_hit / box_hit_exact against the
oracle's boxRayIntersect, src/Lib.hs:798-814, and the joint slab test).

The walks cull with the reference's per-axis test AND a joint slab test, decided without divisions
(`box_hit`: products with RN(1/d), a rounding band, an exact fall-back). These records check that
decision against the same test with IEEE divisions and against the oracle, bit for bit, on:
random boxes and rays; rays with zero direction components (the Lambertian quirk's (1, 0, 0)), the
origin inside, outside and on a zero axis's slab planes; NaN and infinite bounds; and a slab product
that overflows where the quotient is still finite (coordinates near DBL_MAX: the product's infinity is
not the quotient, so the test must fall back rather than reject). Parity is exact.
"""
import numpy as np
import pytest

import pyoracle
import rtamd

MAX = np.finfo(np.float64).max


def overflow_records(n, seed=5):
    """Boxes whose lower x slab quotient is finite just below DBL_MAX while f * RN(1/d) overflows (the
    upper slab's quotient is +inf itself); the ray runs along +x from the origin (y, z zero: those slabs
    constrain nothing), t_max = inf. The reference's test accepts them."""
    rng = np.random.default_rng(seed)
    recs = []
    with np.errstate(over="ignore"):
        for _ in range(200000):
            d = rng.uniform(0.5, 1.0)
            f0 = MAX * d
            for _ in range(8):
                if np.isfinite(f0 / d):
                    break
                f0 = np.nextafter(f0, 0.0)
            if np.isfinite(f0 / d) and np.isinf(f0 * (1.0 / d)):
                recs.append([f0, -1.0, -1.0, MAX, 1.0, 1.0, 0.0, 0.0, 0.0, d, 0.0, 0.0, 1e-3, np.inf])
                if len(recs) == n:
                    break
    assert len(recs) == n
    return np.array(recs)


def random_records(n, seed=11):
    rng = np.random.default_rng(seed)
    lo = rng.uniform(-5, 5, (n, 3))
    hi = lo + rng.uniform(0, 4, (n, 3))
    o = rng.uniform(-8, 8, (n, 3))
    d = rng.normal(size=(n, 3))
    # zero direction components (one or two axes), origins on slab planes, exact-face t bounds
    z = rng.random((n, 3)) < 0.25
    d[z] = 0.0
    on = rng.random((n, 3)) < 0.1
    o[on] = np.where(rng.random(on.sum()) < 0.5, lo[on], hi[on])
    tmin = np.full(n, 1e-3)
    tmax = np.where(rng.random(n) < 0.5, np.inf, rng.uniform(0, 20, n))
    tmax[rng.random(n) < 0.05] = np.nan           # a rect hit at t = NaN as the bound (src/Lib.hs:1014-1028)
    far = rng.random(n) < 0.05                    # huge coordinates (2^120 .. 2^1000)
    o[far] *= 2.0 ** rng.uniform(120, 1000, (far.sum(), 1))
    return np.column_stack([lo, hi, o, d, tmin, tmax])


def _scene():
    sc, _ = rtamd.make_scene("three_spheres", rtamd.randGen(1))
    return sc


def test_oracle_box_probe():
    """The oracle: the overflow records pass the reference's test; joint implies per-axis."""
    sc = _scene()
    out = pyoracle.probe(sc, "box", overflow_records(8))
    assert (out == 1.0).all()
    out = pyoracle.probe(sc, "box", random_records(4000))
    assert np.array_equal(out[:, 0], out[:, 1])
    assert not ((out[:, 0] == 1) & (out[:, 2] == 0)).any()
    assert 0.05 < out[:, 2].mean() < 0.95


def _far(recs):
    """Records whose box has a finite coordinate beyond 2^100: in a world holding such a box the walks
    take the reference's per-axis test alone (rt_render.hip far_boxes, RT_FLAG_REFERENCE_CULL)."""
    box = recs[:, :6]
    return (np.isfinite(box) & (np.abs(box) > 2.0 ** 100)).any(axis=1)


@pytest.mark.gpu
def test_device_box_test_matches_oracle(gpu_ctx):
    sc = _scene()
    gpu_ctx.upload(sc)
    recs = np.vstack([random_records(20000), overflow_records(16)])
    far = _far(recs)
    assert far.sum() == 16
    dev = gpu_ctx.probe("box", recs)
    ref = pyoracle.probe(sc, "box", recs)
    # with divisions: both tests bit for bit; the walks' test: the joint one within 2^100, else per-axis
    walks = np.where(far, dev[:, 2], dev[:, 0])
    bad = np.nonzero((dev[:, 1:] != ref[:, 1:]).any(axis=1) | (walks != np.where(far, ref[:, 2], ref[:, 0])))[0]
    assert bad.size == 0, (bad[:5], recs[bad[:5]], dev[bad[:5]], ref[bad[:5]])
    assert (ref[far] == 1.0).all()
    # (inside 2^100 the division-free test never needs the rule: its infinities are zero axes' quotients)
    assert np.array_equal(dev[~far, 0], ref[~far, 0])


@pytest.mark.gpu
def test_far_box_world_walks_the_per_axis_test(gpu_ctx):
    """A world with a BVH box beyond 2^100 (two spheres at x = 1e120 among 24 ordinary ones) renders
    with the per-axis test over the binary tree: no 4-wide steps, tier A equal to the oracle's."""
    b = rtamd.Builder(rtamd.randGen(7))
    mat = b.lambertian(b.constantColor(0.5, 0.6, 0.7))
    rng = np.random.default_rng(3)
    items = [b.sphere((float(x), 0.3, float(z)), 0.3, mat) for x, z in rng.uniform(-4, 4, (24, 2))]
    items += [b.sphere((1e120, 0.0, 0.0), 1.0, mat), b.sphere((1e120, 4.0, 0.0), 1.0, mat)]
    items.append(b.sphere((0.0, -1000.0, 0.0), 1000.0, mat))
    sc = b.finish(b.makeBVH((0.0, 1.0), items), b.unhittable(), (0.7, 0.8, 1.0))
    gpu_ctx.upload(sc)
    cam = rtamd.camera("random_scene", 64, 40)
    w = gpu_ctx.render_work(cam, rtamd.make_params(64, 40, 4, 10, rtamd.RT_RNG_PHILOX, seed=1024))
    assert w["wide_nodes"] == 0 and w["box_tests"] > 0
    gens = rtamd.column_gens(b.gen, 64)
    p = rtamd.make_params(64, 40, 4, 10, rtamd.RT_RNG_EXACT)
    rgb_g, _, _ = gpu_ctx.render(cam, p, gens)
    rgb_o, _, _, _ = pyoracle.render(sc, cam, p, col_gens=gens, linear=False)
    assert np.array_equal(rgb_g, rgb_o)

"""CPU replica of the device's division-free box test (rt_trace.h box_hit) against the reference's
exact per-axis test plus the joint slab filter (box_hit_exact; boxRayIntersect, src/Lib.hs:798-814):
whenever the fast path decides, its answer must equal the exact test's. Rays include zero direction
components (the Lambertian quirk's (1, 0, 0), round 4), origins on slab planes, huge and tiny values.
numpy float64 is IEEE binary64 like the device's fp64 (no FMA involved here); np.fmin / np.fmax drop
a NaN operand as the device's v_min_f64 / v_max_f64 (IEEE minNum / maxNum) do."""
import numpy as np


def in_range(x):
    ax = np.abs(x)
    return (ax >= 2.0 ** -900) & (ax <= 2.0 ** 900)


def gmax(x, y):  # GHC Ord default: if x <= y then y else x
    return np.where(x <= y, y, x)


def gmin(x, y):
    return np.where(x <= y, x, y)


def exact(lo, hi, o, d, t_min, t_max):
    """box_hit_exact(joint = true): the reference's per-axis test AND the joint slab test."""
    ok = np.ones(len(o), dtype=bool)
    lmax, hmin = t_min.copy(), t_max.copy()
    with np.errstate(all="ignore"):
        for a in range(3):
            ta = (lo[:, a] - o[:, a]) / d[:, a]
            tb = (hi[:, a] - o[:, a]) / d[:, a]
            lt = ta < tb
            t0, t1 = np.where(lt, ta, tb), np.where(lt, tb, ta)
            lo_a, hi_a = gmax(t0, t_min), gmin(t1, t_max)
            ok &= hi_a > lo_a
            lmax = np.where(lo_a > lmax, lo_a, lmax)
            hmin = np.where(hi_a < hmin, hi_a, hmin)
    return ok & (hmin > lmax)


def fast(lo, hi, o, d, t_min, t_max):
    """box_hit's division-free decision: (decided, answer)."""
    with np.errstate(all="ignore"):
        inv = 1.0 / d
        safe = np.ones(len(o), dtype=bool)
        for a in range(3):
            safe &= (d[:, a] == 0.0) | in_range(d[:, a])
            safe &= np.abs(o[:, a]) <= 2.0 ** 100
        L, U = t_min.copy(), t_max.copy()
        nan = np.zeros(len(o), dtype=bool)
        for a in range(3):
            ta = (lo[:, a] - o[:, a]) * inv[:, a]
            tb = (hi[:, a] - o[:, a]) * inv[:, a]
            nan |= np.isnan(ta) | np.isnan(tb)
            L = np.fmax(L, np.fmin(ta, tb))
            U = np.fmin(U, np.fmax(ta, tb))
        band = 2.0 ** -48 * (np.abs(L) + np.abs(U))
        ok_band = (band > 2.0 ** -1000) & (band < np.inf)
        ok = safe & ~nan
        yes = ok & ok_band & (U - L > band)
        no = ok & ((ok_band & (L - U > band)) | (L == np.inf) | (U == -np.inf))
    return yes | no, yes


def _rays(rng, n):
    lo = rng.uniform(-50, 50, (n, 3))
    hi = lo + rng.exponential(5, (n, 3))
    o = rng.uniform(-80, 80, (n, 3))
    d = rng.normal(0, 1, (n, 3))
    # zero components (the quirk's axis directions), sometimes both signs of zero
    z = rng.random((n, 3)) < 0.3
    d[z] = np.where(rng.random(z.sum()) < 0.5, 0.0, -0.0)
    # origins exactly on slab planes, inside slabs of zero axes, far away; scaled directions
    on = rng.random((n, 3)) < 0.1
    o[on] = np.where(rng.random(on.sum()) < 0.5, lo[on], hi[on])
    d *= rng.choice([1.0, 1e-3, 600.0, 1e-200, 1e200], (n, 1), p=[0.6, 0.1, 0.2, 0.05, 0.05])
    t_min = np.full(n, 1e-4)
    t_max = np.where(rng.random(n) < 0.3, np.inf, rng.exponential(50, n))
    # a bound exactly at a slab distance now and then
    return lo, hi, o, d, t_min, t_max


def test_fast_decisions_equal_the_exact_test():
    rng = np.random.default_rng(2026)
    decided_total = 0
    for _ in range(20):
        lo, hi, o, d, t_min, t_max = _rays(rng, 200_000)
        dec, ans = fast(lo, hi, o, d, t_min, t_max)
        ref = exact(lo, hi, o, d, t_min, t_max)
        bad = dec & (ans != ref)
        assert not bad.any(), (lo[bad][:3], hi[bad][:3], o[bad][:3], d[bad][:3], t_max[bad][:3])
        decided_total += dec.sum()
    assert decided_total > 0.9 * 20 * 200_000  # (the exact fall-back stays rare)


def test_quirk_direction_is_decided_without_divisions():
    """d = (1, 0, 0): every box is decided by the fast path unless the origin lies on a y or z slab plane."""
    rng = np.random.default_rng(7)
    n = 100_000
    lo = rng.uniform(-50, 50, (n, 3))
    hi = lo + rng.exponential(5, (n, 3))
    o = rng.uniform(-80, 80, (n, 3))
    d = np.tile([1.0, 0.0, 0.0], (n, 1))
    t_min, t_max = np.full(n, 1e-4), rng.exponential(50, n)
    dec, ans = fast(lo, hi, o, d, t_min, t_max)
    assert dec.mean() > 0.999
    assert (ans[dec] == exact(lo, hi, o, d, t_min, t_max)[dec]).all()


def test_far_boxes_are_left_to_the_per_axis_test():
    """Why the host walks a world with a finite box coordinate beyond 2^100 with the per-axis test
    (rt_render.hip far_boxes): there a slab product can overflow while the quotient is finite, and the
    fast path would read the product's +inf as the quotient (a false reject). Within 2^100
    (and |o| <= 2^100, ray_safe) a product over a non-zero axis stays below 2^1001."""
    import test_box_probe as bp
    r = bp.overflow_records(8)
    lo, hi, o, d, t_min, t_max = r[:, 0:3], r[:, 3:6], r[:, 6:9], r[:, 9:12], r[:, 12], r[:, 13]
    dec, ans = fast(lo, hi, o, d, t_min, t_max)
    assert (dec & ~ans).all() and exact(lo, hi, o, d, t_min, t_max).all()
    rng = np.random.default_rng(9)
    n = 200_000
    lo = rng.uniform(-1, 1, (n, 3)) * 2.0 ** 100
    hi = np.minimum(lo + rng.uniform(0, 2, (n, 3)) * 2.0 ** 99, 2.0 ** 100)
    o = rng.uniform(-1, 1, (n, 3)) * 2.0 ** 100
    d = rng.choice([-1.0, 1.0], (n, 3)) * 2.0 ** -900 * rng.uniform(1, 1.001, (n, 3))
    with np.errstate(over="ignore"):
        assert np.isfinite((lo - o) * (1.0 / d)).all() and np.isfinite((hi - o) * (1.0 / d)).all()
    dec, ans = fast(lo, hi, o, d, np.full(n, 1e-4), np.full(n, np.inf))
    assert (ans[dec] == exact(lo, hi, o, d, np.full(n, 1e-4), np.full(n, np.inf))[dec]).all()

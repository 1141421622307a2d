"""Statistics for comparing two Monte-Carlo renders of the same frame as distributions (tier A, the
reference's per-column SplitMix streams and medium semantics, against tier B, the per-(pixel, sample)
Philox streams with keyed medium draws: tests/test_gpu_tiers.py, tests/test_tier_stats.py).

Both renders estimate the same per-pixel expectation when tier B's draws are independent uniforms in
the places the reference draws them. The pixel differences d = A - B then have mean 0, and pixels are
independent (tier B: one stream per pixel and sample; tier A: one stream per column, whose successive
pixels draw successive, independent numbers), so the mean of d over a block of n pixels, divided by
its sample standard error sd(d) / sqrt(n), is ~ N(0, 1) for n in the hundreds. The reference's
Lambertian light-mixture quirk (src/Lib.hs:829-835) makes many samples NaN; those
renders use RT_FLAG_NAN_ZERO (the finite part of every sample, the same estimator on both sides), and
the NaN probability is compared separately on one-sample renders (a pixel is NaN iff its one sample
is): per block, a two-proportion z with the pooled proportion."""
import numpy as np


def _blocks(x, block):
    H, W = x.shape[:2]
    hb, wb = H // block, W // block
    x = x[: hb * block, : wb * block]
    return x.reshape(hb, block, wb, block, *x.shape[2:])


def mean_z(a, b, block):
    """Per-block z of the mean pixel difference (a, b: H x W x C finite renders) and the whole frame's z per
    channel. A block whose differences are all equal (sd 0: e.g. both tiers black or background there) has z 0
    when the difference is 0, else +-inf."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = a - b
    # (differences at the rounding level are the two summation orders of one value — e.g. a sky pixel whose
    # every sample is the background: tier A sums its samples in one chain, tier B in chunks — not noise)
    d = np.where(np.abs(d) <= 1e-12 * np.maximum(np.abs(a), np.abs(b)), 0.0, d)
    db = _blocks(d, block)
    n = block * block
    m = db.mean(axis=(1, 3))
    sd = db.std(axis=(1, 3), ddof=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(sd > 0, m / (sd / np.sqrt(n)), np.where(m == 0, 0.0, np.copysign(np.inf, m)))
        flat = d.reshape(-1, d.shape[-1])
        sdg = flat.std(axis=0, ddof=1)
        zg = np.where(sdg > 0, flat.mean(axis=0) / (sdg / np.sqrt(flat.shape[0])), 0.0)
    return z, zg


def nan_z(nan_a, nan_b, block):
    """Per-block two-proportion z of the NaN fraction (nan_a, nan_b: H x W booleans), and the whole frame's."""
    pa = _blocks(np.asarray(nan_a, dtype=np.float64), block).mean(axis=(1, 3))
    pb = _blocks(np.asarray(nan_b, dtype=np.float64), block).mean(axis=(1, 3))
    n = block * block

    def z2(pa, pb, n):
        p = (pa + pb) / 2
        se = np.sqrt(p * (1 - p) * 2 / n)
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(se > 0, (pa - pb) / se, 0.0)

    N = np.asarray(nan_a).size
    return z2(pa, pb, n), float(z2(np.mean(nan_a), np.mean(nan_b), N)), float(np.mean(nan_a)), float(np.mean(nan_b))


def summary(lin_a, lin_b, nan_a, nan_b, block):
    """The statistics one scene's comparison reports."""
    z, zg = mean_z(lin_a, lin_b, block)
    zn, zng, fa, fb = nan_z(nan_a, nan_b, block)
    return {"max_abs_z_block_mean": float(np.max(np.abs(z))), "z_frame_mean": [float(x) for x in zg],
            "max_abs_z_block_nan": float(np.max(np.abs(zn))), "z_frame_nan": zng, "nan_frac": (fa, fb),
            "blocks": int(z.shape[0] * z.shape[1]),
            "frame_mean": (np.asarray(lin_a).reshape(-1, 3).mean(0).tolist(),
                           np.asarray(lin_b).reshape(-1, 3).mean(0).tolist())}

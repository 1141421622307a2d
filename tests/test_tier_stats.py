"""CPU: the tier-A/tier-B distribution statistics (tests/tier_stats.py) — calibrated on synthetic renders
(null: |z| stays small; a 2 % bias or a shifted NaN rate is caught) — and the oracle's own tier B against
its tier A (the reference's stream layout and medium semantics, src/Lib.hs:1053-1080, 1491-1523) on the
media worlds at sizes the CPU finishes in seconds. The GPU runs the same comparison at larger sizes
(tests/test_gpu_tiers.py)."""
import os

import numpy as np
import pytest

import pyoracle
import rtamd
from tier_stats import mean_z, nan_z, summary

EARTH = os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz")


def test_statistics_calibrated_on_synthetic_renders():
    rng = np.random.default_rng(3)
    H, W, spp = 256, 256, 16
    truth = rng.uniform(0.05, 0.5, (H, W, 3))

    def render(bias=0.0):  # per-pixel average of spp exponential samples (heavy-ish tails)
        return truth * (1 + bias) * rng.exponential(1.0, (H, W, 3, spp)).mean(-1)

    z, zg = mean_z(render(), render(), 16)
    assert np.abs(z).max() < 4.5 and np.abs(zg).max() < 4.0
    z, zg = mean_z(render(0.02), render(), 16)
    assert np.abs(zg).min() > 6  # a 2 % bias over the frame
    na, nb = rng.random((H, W)) < 0.3, rng.random((H, W)) < 0.3
    zn, zng, _, _ = nan_z(na, nb, 16)
    assert np.abs(zn).max() < 4.5 and abs(zng) < 4.0
    zn, zng, _, _ = nan_z(rng.random((H, W)) < 0.32, nb, 16)
    assert abs(zng) > 4
    # degenerate blocks: identical renders give z = 0, never NaN
    same = render()
    z, zg = mean_z(same, same, 16)
    assert (z == 0).all() and (zg == 0).all()


@pytest.mark.parametrize("name,camname,W,H,spp", [("cornell_smoke", "cornell", 96, 96, 12),
                                                  ("next_week_final", "next_week", 96, 96, 4),
                                                  ("random", "random_scene", 128, 80, 6)])
def test_oracle_tier_b_matches_tier_a_in_distribution(name, camname, W, H, spp):
    earth = np.load(EARTH)["rgb"] if name in ("random", "next_week_final") else None
    sc, g1 = rtamd.make_scene(name, rtamd.randGen(1024), earth=earth)
    cam = rtamd.camera(camname, W, H)
    gens = rtamd.column_gens(g1, W)
    Z = rtamd.RT_FLAG_NAN_ZERO
    _, lin_a, _, _ = pyoracle.render(sc, cam, rtamd.make_params(W, H, spp, 50, rtamd.RT_RNG_EXACT, flags=Z), col_gens=gens)
    _, lin_b, _, _ = pyoracle.render(sc, cam, rtamd.make_params(W, H, spp, 50, rtamd.RT_RNG_PHILOX, seed=1024, flags=Z))
    assert np.isfinite(lin_a).all() and np.isfinite(lin_b).all()
    _, n_a, _, _ = pyoracle.render(sc, cam, rtamd.make_params(W, H, 1, 50, rtamd.RT_RNG_EXACT),
                                   col_gens=rtamd.column_gens(g1, W, seed=50_000))
    _, n_b, _, _ = pyoracle.render(sc, cam, rtamd.make_params(W, H, 1, 50, rtamd.RT_RNG_PHILOX, seed=77))
    s = summary(lin_a, lin_b, np.isnan(n_a).any(axis=2), np.isnan(n_b).any(axis=2), 16)
    print(f"oracle tiers {name} {W}x{H}x{spp}: {s}")
    assert s["frame_mean"][0][0] > 0
    assert s["max_abs_z_block_mean"] <= 5.5 and max(abs(z) for z in s["z_frame_mean"]) <= 4.5
    assert s["max_abs_z_block_nan"] <= 5.5 and abs(s["z_frame_nan"]) <= 4.5

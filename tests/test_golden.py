"""Committed golden vectors (tests/golden/oracle_goldens.npz, made by make_oracle_goldens.py).

CPU: the oracle and the product's host RNG reproduce them bit for bit (a regression pin of the
checker itself). GPU: the HIP path, through the C ABI, matches them with the north-star tolerance
(1e-3 per channel on the displayed float for >= 99.9 % of channels, >= 99.9 % equal bytes) and
exactly in the integer outputs (tier-A end-of-stream generators, closest-hit primitive choice).
The vectors are self-generated (no GHC exists to produce reference ones: SURVEY.md 8c).
"""
import os

import numpy as np
import pytest

import pyoracle
import rtamd
from conftest import parity

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_goldens.npz"))
ROWS = G["c1b_lin"].shape[0]


def _c1():
    sc, g1 = rtamd.make_scene("three_spheres", rtamd.randGen(1024))
    return sc, g1, rtamd.camera("random_scene", 200, 100)


def _cornell():
    sc, g1 = rtamd.make_scene("cornell", rtamd.randGen(1024))
    return sc, g1, rtamd.camera("cornell", 64, 64)


# ------------------------------------------------------------------ CPU: pin the checker
def test_rng_words_and_draws():
    words, _ = pyoracle.words(rtamd.randGen(1024), 32)
    assert np.array_equal(np.array(words, dtype=np.uint64), G["rng_words"])
    g, ours = rtamd.randGen(1024), []
    for _ in range(32):
        x, g = rtamd.randomDouble(g)
        ours.append(x)
    assert np.array_equal(np.array(ours), G["rng_draws"])


def test_oracle_config1_tier_b_golden():
    sc, _, cam = _c1()
    rgb, lin, _, _ = pyoracle.render(sc, cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_PHILOX, seed=1024))
    assert np.array_equal(rgb, G["c1b_rgb"])
    assert np.array_equal(lin[:ROWS], G["c1b_lin"], equal_nan=True)


def test_oracle_config1_tier_a_golden():
    sc, g1, cam = _c1()
    gens = rtamd.column_gens(g1, 200)
    assert np.array_equal(gens, G["c1a_gens_in"])
    rgb, lin, go, _ = pyoracle.render(sc, cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_EXACT), col_gens=gens)
    assert np.array_equal(rgb, G["c1a_rgb"]) and np.array_equal(go, G["c1a_gens_out"])
    assert np.array_equal(lin[:ROWS], G["c1a_lin"], equal_nan=True)


def test_oracle_cornell_tier_a_golden():
    sc, g1, cam = _cornell()
    gens = rtamd.column_gens(g1, 64)
    rgb, lin, go, _ = pyoracle.render(sc, cam, rtamd.make_params(64, 64, 16, 50, rtamd.RT_RNG_EXACT), col_gens=gens)
    assert np.array_equal(rgb, G["cba_rgb"]) and np.array_equal(go, G["cba_gens_out"])
    assert np.array_equal(lin, G["cba_lin"], equal_nan=True)


@pytest.mark.parametrize("name", ["random_book_one", "cornell"])
def test_oracle_closest_hits_golden(name):
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024))
    out = pyoracle.closest_hits(sc, G[f"hits_{name}_rays"], 1e-4, np.inf, seed=3)
    assert np.array_equal(out, G[f"hits_{name}"])


# ------------------------------------------------------------------ GPU: the HIP path against them
def _check_image(rgb, lin, key):
    lin_g = G[f"{key}_lin"]
    ok, eq, dmax = parity(lin[: lin_g.shape[0]], lin_g, rgb, G[f"{key}_rgb"])
    print(f"{key}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, max |d| {dmax:.3g}")
    assert ok >= 0.999, f"{key}: {ok:.5f} of channels within 1e-3 (max |d| {dmax:.3g})"
    assert eq >= 0.999, f"{key}: {eq:.5f} of bytes equal"


@pytest.mark.gpu
def test_gpu_config1_tier_b_golden(gpu_ctx):
    sc, _, cam = _c1()
    gpu_ctx.upload(sc)
    rgb, lin, _ = gpu_ctx.render(cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_PHILOX, seed=1024), linear=True)
    _check_image(rgb, lin, "c1b")


@pytest.mark.gpu
def test_gpu_config1_tier_a_golden(gpu_ctx):
    sc, _, cam = _c1()
    gpu_ctx.upload(sc)
    rgb, lin, go = gpu_ctx.render(cam, rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_EXACT),
                                  G["c1a_gens_in"], linear=True, want_gens=True)
    _check_image(rgb, lin, "c1a")
    print(f"c1a: end generators equal in {(go == G['c1a_gens_out']).all(axis=1).mean():.6f} of columns")
    assert np.array_equal(go, G["c1a_gens_out"])


@pytest.mark.gpu
def test_gpu_cornell_tier_a_golden(gpu_ctx):
    sc, _, cam = _cornell()
    gpu_ctx.upload(sc)
    rgb, lin, go = gpu_ctx.render(cam, rtamd.make_params(64, 64, 16, 50, rtamd.RT_RNG_EXACT),
                                  G["cba_gens_in"], linear=True, want_gens=True)
    _check_image(rgb, lin, "cba")
    print(f"cba: end generators equal in {(go == G['cba_gens_out']).all(axis=1).mean():.6f} of columns")
    assert np.array_equal(go, G["cba_gens_out"])


@pytest.mark.gpu
@pytest.mark.parametrize("walk", [0, rtamd.RT_DEBUG_RESUMABLE, rtamd.RT_DEBUG_WIDE])
@pytest.mark.parametrize("name", ["random_book_one", "cornell"])
def test_gpu_closest_hits_golden(gpu_ctx, name, walk):
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024))
    gpu_ctx.upload(sc)
    got = gpu_ctx.closest_hits(G[f"hits_{name}_rays"], 1e-4, np.inf, seed=3, flags=walk)
    ref = G[f"hits_{name}"]
    exact = [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]  # hit, t, p, normal, frontFace, material: bit-identical
    assert np.array_equal(got[:, exact], ref[:, exact])
    du = np.abs(got[:, 8:10] - ref[:, 8:10])  # sphere u, v go through OCML vs glibc atan/asin
    du[np.isnan(got[:, 8:10]) & np.isnan(ref[:, 8:10])] = 0
    assert np.all(du <= 2e-15)

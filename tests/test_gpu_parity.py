"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Tolerance (BASELINE.json north_star): 1e-3 per channel on the displayed float, for >= 99.9 % of
channels; both sides fp64, same RNG streams. The residue, if any, comes from fp64
transcendental implementations (OCML on the GPU vs glibc in the oracle) flipping a branch.
Integer outputs (tier-A end-of-stream generators) must match exactly.
"""
import numpy as np
import pytest

import bench
import pyoracle
import rtamd
from conftest import parity

pytestmark = pytest.mark.gpu


def _scene(name, **kw):
    return rtamd.make_scene(name, rtamd.randGen(1024), **kw)


def _cmp(ctx, scene, cam, params, col_gens=None, frac=0.999, what=""):
    ctx.upload(scene)
    rgb_g, lin_g, gens_g = ctx.render(cam, params, col_gens, linear=True, want_gens=col_gens is not None)
    rgb_o, lin_o, gens_o, _ = pyoracle.render(scene, cam, params, col_gens=col_gens)
    ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
    print(f"{what} {params.width}x{params.height}x{params.spp}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, "
          f"max |d| {dmax:.3g}")
    assert ok >= frac, f"only {ok:.5f} of channels within 1e-3 (max |d| {dmax:.3g})"
    assert eq >= frac, f"only {eq:.5f} of bytes equal"
    return rgb_g, lin_g, gens_g, gens_o


def test_config1_tier_b(gpu_ctx):
    """Config 1 (200x100, 10 spp, depth 10), Philox streams."""
    sc, _ = _scene("three_spheres")
    cam = rtamd.camera("random_scene", 200, 100)
    p = rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_PHILOX, seed=1024)
    _cmp(gpu_ctx, sc, cam, p)


def test_config1_tier_a_exact_stream(gpu_ctx):
    """Config 1 with the reference's own stream layout: one SplitMix generator per column."""
    sc, g1 = _scene("three_spheres")
    cam = rtamd.camera("random_scene", 200, 100)
    gens = rtamd.column_gens(g1, 200)
    p = rtamd.make_params(200, 100, 10, 10, rtamd.RT_RNG_EXACT)
    _, _, gens_g, gens_o = _cmp(gpu_ctx, sc, cam, p, col_gens=gens, what="config1 tier A")
    # every column consumed exactly the same number of draws (integers: exact)
    print(f"tier-A end generators equal: {(gens_g == gens_o).all(axis=1).mean():.6f} of columns")
    assert np.array_equal(gens_g, gens_o)


def test_book_one_tier_b(gpu_ctx):
    sc, _ = _scene("random_book_one")
    cam = rtamd.camera("random_scene", 120, 80)
    p = rtamd.make_params(120, 80, 4, 50, rtamd.RT_RNG_PHILOX, seed=7)
    _cmp(gpu_ctx, sc, cam, p)


@pytest.mark.parametrize("w,h,spp,ch", [(32, 24, 33, 1), (64, 64, 600, 3), (80, 96, 1200, 9), (256, 256, 130, 8),
                                        (160, 120, 2200, 18)])
def test_tier_b_sample_chunks(gpu_ctx, w, h, spp, ch):
    """A pixel's samples are summed per chunk (rt_sample_chunk: the fill-limited 1, 3, 9 and the
    8-sample floor and ceil(spp/128) branches at 8 and 18), chunk sums in chunk order — the device's
    work-items, combined by `combine_chunks` — exactly as the oracle. The last two use config 1's
    scene at depth 10 with RT_FLAG_NAN_ZERO, so that every sample's finite colour is summed (cheap
    for the oracle; the light-mixture quirk would make most pixels NaN)."""
    assert bench.sample_chunk(w * h, spp) == ch
    cheap = w * h * spp > 4_000_000
    sc, _ = _scene("three_spheres" if cheap else "random_book_one")
    cam = rtamd.camera("random_scene", w, h)
    p = rtamd.make_params(w, h, spp, 10 if cheap else 50, rtamd.RT_RNG_PHILOX, seed=3,
                          flags=rtamd.RT_FLAG_NAN_ZERO if cheap else 0)
    rgb_g, lin_g, _, _ = _cmp(gpu_ctx, sc, cam, p, what=f"chunks of {ch}")
    rgb_o, lin_o, _, _ = pyoracle.render(sc, cam, p)
    close = np.isclose(lin_g, lin_o, rtol=1e-12, atol=0, equal_nan=True).mean()
    print(f"chunks of {ch}: linear within 1e-12 relative {close:.6f}")
    assert close >= 0.99, close


def test_cornell_tier_b(gpu_ctx):
    sc, _ = _scene("cornell")
    cam = rtamd.camera("cornell", 64, 64)
    p = rtamd.make_params(64, 64, 8, 50, rtamd.RT_RNG_PHILOX, seed=1024)
    _cmp(gpu_ctx, sc, cam, p)


def test_cornell_tier_a(gpu_ctx):
    sc, g1 = _scene("cornell")
    cam = rtamd.camera("cornell", 48, 48)
    gens = rtamd.column_gens(g1, 48)
    p = rtamd.make_params(48, 48, 4, 50, rtamd.RT_RNG_EXACT)
    _, _, gens_g, gens_o = _cmp(gpu_ctx, sc, cam, p, col_gens=gens, what="cornell tier A")
    print(f"tier-A end generators equal: {(gens_g == gens_o).all(axis=1).mean():.6f} of columns")
    assert np.array_equal(gens_g, gens_o)


@pytest.mark.parametrize("name,camname,w,h,spp", [
    ("cornell_smoke", "cornell", 40, 40, 4),        # ConstantMedium draws inside the walk (Lib.hs:1053-1080)
    ("next_week_final", "next_week", 48, 48, 3),    # media, motion blur, Perlin marble, the earth raster
    ("random", "random_scene", 64, 40, 3),          # moving spheres: the time draw (Lib.hs:1106-1108, 1253-1267)
    ("random_book_one", "random_scene", 80, 48, 4),  # the bench scene (C2)
    ("two_perlin_spheres", "two_spheres", 48, 32, 4),
    ("earth", "two_spheres", 48, 32, 4),
    ("simple_light", "two_spheres", 48, 32, 4)])
def test_tier_a_rng_consuming_features(gpu_ctx, name, camname, w, h, spp):
    """Tier A (RT_RNG_EXACT, the drop-in runRenderAMD's mode: the reference's per-column SplitMix streams)
    against the oracle on every feature that consumes draws: medium draws interleaved with the walk
    (Lib.hs:1053-1080), the motion-blur time draw (Lib.hs:1253-1267, 1106-1108), Isotropic's rejection
    draws (Lib.hs:861-865), Perlin and image textures.
    1. RT_FLAG_SHARED_LIBM (both sides evaluate sin/cos/log/atan/asin in include/rt_libm.h): bytes and
       end-of-stream generators identical on every scene, linear averages within the tolerance (the device
       accumulates the path's throughput forwards, the oracle in the reference's continuation order:
       rounding only).
    2. Each side's own libm (OCML on the device, glibc in the oracle): the north-star tolerance and equal
       end generators, except where a column's serial stream meets a libm ulp that later flips a branch
       (next_week_final: thousands of fog bounces per column). There the columns that consumed the same
       draws (equal end generators) must match to the tolerance, and the oracle with glibc against the
       oracle with rt_libm.h diverges in the same way: a libm property, not a device one."""
    earth = np.load(_earth_path())["rgb"] if name in ("earth", "random", "next_week_final") else None
    sc, g1 = _scene(name, earth=earth)
    cam = rtamd.camera(camname, w, h)
    gens = rtamd.column_gens(g1, w)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(w, h, spp, 50, rtamd.RT_RNG_EXACT, flags=rtamd.RT_FLAG_SHARED_LIBM)
    rgb_g, lin_g, gens_g = gpu_ctx.render(cam, p, gens, linear=True, want_gens=True)
    rgb_o, lin_o, gens_o, _ = pyoracle.render(sc, cam, p, col_gens=gens)
    ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
    print(f"{name} tier A, shared libm: bytes equal {eq:.6f}, channels within 1e-3 {ok:.6f}, max |d| {dmax:.3g}, "
          f"end generators equal {float((gens_g == gens_o).all(axis=1).mean()):.6f}")
    assert np.array_equal(gens_g, gens_o) and np.array_equal(rgb_g, rgb_o) and ok == 1.0
    p = rtamd.make_params(w, h, spp, 50, rtamd.RT_RNG_EXACT)
    rgb_g, lin_g, gens_g = gpu_ctx.render(cam, p, gens, linear=True, want_gens=True)
    rgb_o, lin_o, gens_o, _ = pyoracle.render(sc, cam, p, col_gens=gens)
    ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
    same_cols = (gens_g == gens_o).all(axis=1)
    print(f"{name} tier A, device libm vs glibc: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, max |d| "
          f"{dmax:.3g}, end generators equal in {same_cols.mean():.6f} of columns")
    if name != "next_week_final":
        assert ok >= 0.999 and eq >= 0.999 and same_cols.all()
        return
    ok_c, eq_c, _ = parity(lin_g[:, same_cols], lin_o[:, same_cols], rgb_g[:, same_cols], rgb_o[:, same_cols])
    ps = rtamd.make_params(w, h, spp, 50, rtamd.RT_RNG_EXACT, flags=rtamd.RT_FLAG_SHARED_LIBM)
    rgb_s, lin_s, gens_s, _ = pyoracle.render(sc, cam, ps, col_gens=gens)
    ok_l, eq_l, _ = parity(lin_s, lin_o, rgb_s, rgb_o)
    print(f"  columns with equal end generators: channels within 1e-3 {ok_c:.6f}, bytes equal {eq_c:.6f}; oracle "
          f"glibc vs rt_libm.h: channels within 1e-3 {ok_l:.6f}, end generators equal in "
          f"{(gens_s == gens_o).all(axis=1).mean():.6f} of columns")
    # measured (rounds 5-6, deterministic on a given device libm): 47 of 48 columns keep the glibc draw count at
    # 48x48x3; the bound allows one more column to diverge (~2.5e-5 divergences per sample on
    # this scene, none on Cornell or book one at their full bench frames)
    assert same_cols.mean() >= 0.95 and ok_c >= 0.999 and eq_c >= 0.999
    assert (gens_s == gens_o).all(axis=1).mean() < 1.0  # (the libm swap alone diverges columns too)


@pytest.mark.parametrize("name,camname", [("cornell_smoke", "cornell"), ("simple_light", "two_spheres"),
                                          ("two_perlin_spheres", "two_spheres"), ("two_spheres", "two_spheres"),
                                          ("earth", "two_spheres"), ("random", "random_scene"),
                                          ("next_week_final", "next_week")])
def test_scene_library_tier_b(gpu_ctx, name, camname):
    earth = np.load(_earth_path())["rgb"] if name in ("earth", "random", "next_week_final") else None
    sc, _ = _scene(name, earth=earth)
    cam = rtamd.camera(camname, 40, 40)
    p = rtamd.make_params(40, 40, 4, 50, rtamd.RT_RNG_PHILOX, seed=99)
    _cmp(gpu_ctx, sc, cam, p, what=name)


def _earth_path():
    import os
    return os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz")


def _ulp_close(a, b, ulps):
    return np.abs(a - b) <= ulps * np.spacing(np.maximum(np.abs(a), np.abs(b)))


@pytest.mark.parametrize("flags", [0, rtamd.RT_FLAG_REFERENCE_CULL, rtamd.RT_DEBUG_RESUMABLE])
@pytest.mark.parametrize("name", ["random_book_one", "cornell", "next_week_final", "cornell_smoke"])
def test_closest_hits_bit_exact(gpu_ctx, name, flags):
    """hit over the whole world DAG, by the recursive walk (flags 0 / reference cull) and by the
    render loop's resumable walk (media and instance frames walked in the reference's order,
    records rebuilt through the frames at the end). Surface hits: t, p, normal, frontFace,
    material bit-identical (u, v of spheres go through atan/asin: within 2 ulps). Medium hits: t
    through `log` (OCML vs glibc, <= 1 ulp apart), so t and p within 4 ulps, the rest exact."""
    earth = np.load(_earth_path())["rgb"] if name == "next_week_final" else None
    sc, _ = _scene(name, earth=earth)
    gpu_ctx.upload(sc)
    rng = np.random.default_rng(5)
    n = 1 << 16
    if name == "random_book_one":
        o = np.array([13.0, 2.0, 3.0]) + rng.normal(0, 0.5, (n, 3))
        d = np.array([-13.0, -2.0, -3.0]) + rng.normal(0, 3.0, (n, 3))
    else:
        o = np.array([278.0, 278.0, -800.0]) + rng.normal(0, 20, (n, 3))
        d = rng.normal(0, 1, (n, 3)) + np.array([0, 0, 1.0])
        o[: n // 2] = rng.uniform(20, 530, (n // 2, 3))  # rays from inside the box
    rays = np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)
    got = gpu_ctx.closest_hits(rays, 1e-4, np.inf, seed=3, flags=flags)
    ref = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    assert got[:, 0].sum() > n // 4
    mats = sc.materials
    medium = (ref[:, 0] == 1) & (mats["type"][ref[:, 11].astype(int)] == 4)  # Isotropic phase = medium hit
    exact_cols = [0, 5, 6, 7, 10, 11]
    assert np.array_equal(got[:, exact_cols], ref[:, exact_cols])
    surf = ~medium
    assert np.array_equal(got[surf][:, 1:5], ref[surf][:, 1:5]), "surface t/p not bit-identical"
    gm, rm, ray_m = got[medium], ref[medium], rays[medium]
    assert _ulp_close(gm[:, 1], rm[:, 1], 4).all()
    scale = np.abs(ray_m[:, 0:3]) + np.abs(rm[:, 1:2] * ray_m[:, 3:6])  # p = o + t*d may cancel
    assert (np.abs(gm[:, 2:5] - rm[:, 2:5]) <= 1e-13 * scale).all()
    assert np.all(np.abs(got[:, 8:10] - ref[:, 8:10]) <= 4e-16)
    full = np.all(got == ref, axis=1).mean()
    print(f"{name}: {full:.5f} of rays bit-identical in every field; media hits {int(medium.sum())}")
    assert full >= 0.95


def _special_rays(sc, rng, n):
    """Rays that stress a conservative box test: origins exactly on sphere bounding-box planes,
    axis-aligned directions (exact zeros, both signs: the light-sample direction (1,0,0) of the
    NaN quirk), direction components far below fp32 range, and long grazing rays."""
    nodes = sc.nodes
    sph = nodes[nodes["type"] == rtamd.RT_NODE_SPHERE]
    c = sph["f"][:, :3]
    rad = sph["f"][:, 3]
    k = rng.integers(0, len(sph), n)
    axis = rng.integers(0, 3, n)
    sign = rng.choice([-1.0, 1.0], n)
    o = c[k].copy()
    o[np.arange(n), axis] += sign * rad[k]                      # on the box face (and the sphere)
    o += rng.normal(0, 1, (n, 3)) * (rng.random((n, 1)) < 0.5)  # half of them moved off it
    d = np.zeros((n, 3))
    kind = rng.integers(0, 4, n)
    ax2 = rng.integers(0, 3, n)
    d[np.arange(n), ax2] = rng.choice([-1.0, 1.0], n)           # axis-aligned
    m = kind == 1
    d[m] = rng.normal(0, 1, (m.sum(), 3))
    d[m, ax2[m]] = rng.choice([0.0, -0.0, 1e-40, -1e-300], m.sum())  # one tiny or signed-zero component
    m = kind == 2
    d[m] = np.array([1.0, 0.0, 0.0])                           # htblRandom's Unhittable direction
    m = kind == 3
    d[m] = rng.normal(0, 1, (m.sum(), 3))
    return np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)


@pytest.mark.parametrize("walk", [rtamd.RT_DEBUG_RESUMABLE, rtamd.RT_DEBUG_WIDE, rtamd.RT_DEBUG_QNODE, "w8"])
@pytest.mark.parametrize("name", ["random_book_one", "three_spheres", "cornell", "stress_spheres"])
def test_resumable_walks_closest_hits(gpu_ctx, name, walk, monkeypatch):
    """The render loop's walks (binary resumable; 4-wide with conservative fp32 child boxes; the same
    over the quantised 64-byte nodes and sphere quadruples of spheres-only worlds; the 8-wide tree as
    4-wide record pairs, RTAMD_W8=1, A/B) give the oracle's closest hits (the reference's makeBVH tree,
    fp64 slab tests) on random and adversarial rays: same primitive, t, p, normal bit-identical."""
    if walk in (rtamd.RT_DEBUG_QNODE, "w8"):
        if name == "cornell":
            pytest.skip("quantised and 8-wide trees are built for spheres-only worlds")
        monkeypatch.setenv("RTAMD_QNODE" if walk == rtamd.RT_DEBUG_QNODE else "RTAMD_W8", "1")  # (read at upload)
        walk = rtamd.RT_DEBUG_QNODE if walk == rtamd.RT_DEBUG_QNODE else rtamd.RT_DEBUG_WIDE
    sc, _ = _scene(name, param=3000 if name == "stress_spheres" else 0)
    gpu_ctx.upload(sc)
    rng = np.random.default_rng(17)
    n = 1 << 15
    if name == "cornell":
        o = rng.uniform(20, 530, (n, 3))
        d = rng.normal(0, 1, (n, 3))
        d[: n // 4] = np.eye(3)[rng.integers(0, 3, n // 4)] * rng.choice([-1.0, 1.0], (n // 4, 1))
        rays = np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)
    else:
        o = np.array([13.0, 2.0, 3.0]) + rng.normal(0, 0.5, (n, 3))
        d = np.array([-13.0, -2.0, -3.0]) + rng.normal(0, 3.0, (n, 3))
        rays = np.concatenate([np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1),
                               _special_rays(sc, rng, n)])
    got = gpu_ctx.closest_hits(rays, 1e-4, np.inf, seed=3, flags=walk)
    ref = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    assert got[:, 0].sum() > len(rays) // 8
    bad = ~np.all(got[:, [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]] == ref[:, [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]], axis=1)
    if bad.any():
        import os
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez(f"gpurun_out/walk_{name}_{walk}.npz", rays=rays[bad], got=got[bad], ref=ref[bad])
    assert not bad.any(), f"{int(bad.sum())} of {len(rays)} rays differ"
    du = np.abs(got[:, 8:10] - ref[:, 8:10])  # sphere u, v: OCML vs glibc atan/asin ulps
    du[np.isnan(got[:, 8:10]) & np.isnan(ref[:, 8:10])] = 0  # asin of |y| > 1 by rounding: NaN in both
    assert np.all(du <= 2e-15), f"u/v max |d| {du.max():.3g}"


@pytest.mark.parametrize("name,cam", [("random_book_one", "random_scene"), ("cornell", "cornell"),
                                      ("next_week_final", "next_week"), ("cornell_smoke", "cornell")])
def test_walks_output_identical(gpu_ctx, name, cam, monkeypatch):
    """Full tier-B images: 4-wide walk == binary replacement walk == one-sample-per-lane loop,
    byte for byte and in the linear averages (the walks differ only in which boxes they cull; worlds
    with media or frames take the reference's own order in both loops)."""
    earth = np.load(_earth_path())["rgb"] if name == "next_week_final" else None
    sc, _ = _scene(name, earth=earth)
    c = rtamd.camera(cam, 160, 96)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(160, 96, 4, 50, rtamd.RT_RNG_PHILOX, seed=5)
    monkeypatch.setenv("RTAMD_WIDE", "1")
    rgb_w, lin_w, _ = gpu_ctx.render(c, p, linear=True)
    monkeypatch.setenv("RTAMD_WIDE", "0")
    rgb_b, lin_b, _ = gpu_ctx.render(c, p, linear=True)
    monkeypatch.setenv("RTAMD_BOX_FIRST", "16")  # binary walk: box-only steps while > 16/64 of lanes are at boxes
    rgb_f, lin_f, _ = gpu_ctx.render(c, p, linear=True)
    monkeypatch.setenv("RTAMD_BOX_FIRST", "64")  # (never)
    rgb_n, lin_n, _ = gpu_ctx.render(c, p, linear=True)
    monkeypatch.setenv("RTAMD_REPLACE", "0")
    rgb_s, lin_s, _ = gpu_ctx.render(c, p, linear=True)
    assert np.array_equal(rgb_w, rgb_b) and np.array_equal(rgb_w, rgb_s)
    assert np.array_equal(rgb_w, rgb_f) and np.array_equal(rgb_w, rgb_n)
    assert np.array_equal(lin_w, lin_b, equal_nan=True) and np.array_equal(lin_w, lin_s, equal_nan=True)
    assert np.array_equal(lin_w, lin_f, equal_nan=True) and np.array_equal(lin_w, lin_n, equal_nan=True)
    # media / frame worlds: the mixed walk over 4-wide subtrees == the same walk without them (read at
    # upload: RTAMD_MIXW=0 builds no wide trees)
    monkeypatch.delenv("RTAMD_REPLACE")
    monkeypatch.delenv("RTAMD_BOX_FIRST")
    monkeypatch.setenv("RTAMD_MIXW", "0")
    gpu_ctx.upload(sc)
    rgb_m, lin_m, _ = gpu_ctx.render(c, p, linear=True)
    monkeypatch.delenv("RTAMD_MIXW")
    gpu_ctx.upload(sc)
    assert np.array_equal(rgb_w, rgb_m) and np.array_equal(lin_w, lin_m, equal_nan=True)


def test_shard_invariance(gpu_ctx):
    """Tier B output is byte-identical for any shard count (tiles dealt round-robin)."""
    import ctypes as C
    sc, _ = _scene("random_book_one")
    cam = rtamd.camera("random_scene", 96, 72)
    gpu_ctx.upload(sc)
    base = rtamd.make_params(96, 72, 3, 20, rtamd.RT_RNG_PHILOX, seed=11, tile=16)
    ref, lin_ref, _ = gpu_ctx.render(cam, base, linear=True)
    import torch
    for shards in (2, 3, 8):
        _, _, slab = rtamd.shard_geometry(rtamd.make_params(96, 72, 3, 20, shard_count=shards, tile=16))
        slabs = torch.zeros((shards, slab, 3), dtype=torch.uint8, device="cuda")
        for r in range(shards):
            p = rtamd.make_params(96, 72, 3, 20, rtamd.RT_RNG_PHILOX, seed=11, tile=16, shard_rank=r,
                                  shard_count=shards)
            gpu_ctx.render_shard_async(cam, p, slabs[r].data_ptr())
            torch.cuda.synchronize()
        img = torch.zeros((72, 96, 3), dtype=torch.uint8, device="cuda")
        p = rtamd.make_params(96, 72, 3, 20, rtamd.RT_RNG_PHILOX, seed=11, tile=16, shard_count=shards)
        gpu_ctx.assemble_async(p, slabs.data_ptr(), img.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(img.cpu().numpy(), ref), f"{shards} shards differ"
    del C


def test_joint_culling_is_output_identical(gpu_ctx):
    """The joint slab filter only prunes: full images with and without it are byte-identical."""
    sc, _ = _scene("random_book_one")
    cam = rtamd.camera("random_scene", 200, 120)
    gpu_ctx.upload(sc)
    a, la, _ = gpu_ctx.render(cam, rtamd.make_params(200, 120, 8, 50, rtamd.RT_RNG_PHILOX, seed=5), linear=True)
    b, lb, _ = gpu_ctx.render(cam, rtamd.make_params(200, 120, 8, 50, rtamd.RT_RNG_PHILOX, seed=5,
                                                     flags=rtamd.RT_FLAG_REFERENCE_CULL), linear=True)
    assert np.array_equal(a, b)
    assert np.array_equal(np.isnan(la), np.isnan(lb)) and np.array_equal(la[~np.isnan(la)], lb[~np.isnan(lb)])


def test_nan_cull_is_output_identical(gpu_ctx):
    sc, _ = _scene("random_book_one")
    cam = rtamd.camera("random_scene", 160, 100)
    gpu_ctx.upload(sc)
    a, _, _ = gpu_ctx.render(cam, rtamd.make_params(160, 100, 16, 50, rtamd.RT_RNG_PHILOX, seed=5))
    b, _, _ = gpu_ctx.render(cam, rtamd.make_params(160, 100, 16, 50, rtamd.RT_RNG_PHILOX, seed=5,
                                                    flags=rtamd.RT_FLAG_NAN_CULL))
    assert np.array_equal(a, b)


def test_cornell_1000spp_tracks_reference_render(gpu_ctx):
    """Statistical pin against the reference's own output: cornellBox1000.png is makeCornellBoxScene
    at 500x500, 1000 spp, depth 50 (app/Main.hs), columns seeded from the clock. The GPU render of
    the same configuration (tier B streams) must agree in 10x10-block means of the 8-bit image
    (tests/golden/cornell1000_blocks.npz): MC noise of a block mean is ~0.6 levels per side."""
    import os
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "cornell1000_blocks.npz"))
    sc, _ = _scene("cornell")
    gpu_ctx.upload(sc)
    cam = rtamd.camera("cornell", 500, 500)
    rgb, _, _ = gpu_ctx.render(cam, rtamd.make_params(500, 500, 1000, 50, rtamd.RT_RNG_PHILOX, seed=1024))
    ours = rgb.astype(np.float64).reshape(50, 10, 50, 10, 3).mean(axis=(1, 3))
    d = np.abs(ours - ref["mean"])
    print(f"cornell 1000 spp vs reference PNG: block |d| mean {d.mean():.3f}, p99 {np.percentile(d, 99):.3f}, "
          f"max {d.max():.3f}; image mean {rgb.reshape(-1, 3).mean(0)} vs {ref['image_mean']}")
    # measured (round 1): image means within 0.013 levels, block |d| mean 0.34, p99 1.47, max 2.9
    assert np.abs(rgb.reshape(-1, 3).mean(0) - ref["image_mean"]).max() < 0.1
    assert d.mean() < 0.5 and np.percentile(d, 99) < 2.5 and d.max() < 5.0


@pytest.mark.parametrize("wide", ["0", "1"])
def test_skewed_spine_world_walks(gpu_ctx, wide, monkeypatch):
    """A world whose SAH rebuild is a deep spine (45 spheres at x = -2^k): rays along the row
    enter the near child at every level with the far one stacked, so the binary walk's LDS stack
    must be sized for 1 + max(child needs) on rebuilt nodes (rt_tree_stack_need). Images from
    the binary (RTAMD_WIDE=0) and 4-wide walks match the oracle."""
    from test_bvh import _spine_scene
    sc = _spine_scene()
    assert rtamd.tree_stack_need(rtamd.rebuilt_scene(sc)) >= 10
    cam = rtamd.newCamera((10.0, 0.05, 0.02), (-1.0, 0.0, 0.0), (0.0, 1.0, 0.0), 8.0, 1.0, 0.0, 10.0, 0.0, 1.0)
    p = rtamd.make_params(48, 48, 4, 8, rtamd.RT_RNG_PHILOX, seed=21)
    monkeypatch.setenv("RTAMD_WIDE", wide)
    _cmp(gpu_ctx, sc, cam, p)



@pytest.mark.parametrize("name,cam", [("random_book_one", "random_scene"), ("next_week_final", "next_week")])
def test_work_claims_do_not_change_the_image(gpu_ctx, name, cam, monkeypatch):
    """Work-items are claimed per wave in batches (RTAMD_BATCH, default 1024, tapering as the frame
    runs out): which lane renders which (pixel, chunk) changes, the chunk sums and their order do
    not, so the image is identical for any batch size, tile order or chunk batching. Every item must be
    rendered exactly once:
    each render follows one with another seed (a dropped item would leave that render's chunk sum
    in the buffer), and the counting build counts every sample."""
    earth = np.load(_earth_path())["rgb"] if name == "next_week_final" else None
    sc, _ = _scene(name, earth=earth)
    c = rtamd.camera(cam, 128, 96)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(128, 96, 24, 50, rtamd.RT_RNG_PHILOX, seed=17)
    other = rtamd.make_params(128, 96, 24, 50, rtamd.RT_RNG_PHILOX, seed=99)
    out = []
    slab_chunk = 128 * 96 * 3 * 8  # one chunk's sums (the 24 chunks of one sample each)
    for b, rev, cap in (("1", "0", 0), ("7", "0", 0), ("256", "0", 0), ("4096", "0", 0), ("256", "1", 0),
                        ("256", "0", 5 * slab_chunk), ("1024", "0", 1)):
        monkeypatch.setenv("RTAMD_BATCH", b)
        monkeypatch.setenv("RTAMD_TILE_REV", rev)  # the slab's tiles last to first: work order only
        # chunk sums bounded per launch: the chunks render in batches (5 of 5 chunks, 24 of 1), folded
        # into running sums in chunk order
        if cap:
            monkeypatch.setenv("RTAMD_PARTIAL_CAP", str(cap))
        else:
            monkeypatch.delenv("RTAMD_PARTIAL_CAP", raising=False)
        gpu_ctx.render(c, other)
        out.append(gpu_ctx.render(c, p, linear=True))
        assert gpu_ctx.last_launch()["chunk_batches"] == ({0: 1, 1: 24}.get(cap, 5))
        assert gpu_ctx.render_work(c, p)["samples"] == 128 * 96 * 24
    for rgb, lin, _ in out[1:]:
        assert np.array_equal(rgb, out[0][0]) and np.array_equal(lin, out[0][1], equal_nan=True)


def test_run_render_zip_truncation(gpu_ctx):
    """runRender zips the generators with each row (src/Lib.hs:1519): fewer generators than
    columns truncate every row to that many pixels (the same bytes as those columns of the full
    render), extra generators are ignored, none gives empty rows."""
    sc, g1 = _scene("three_spheres")
    cam = rtamd.camera("random_scene", 48, 24)
    env = rtamd.mkRenderStaticEnv(sc, cam, (48, 24), 3, 10)
    gens = [tuple(int(v) for v in g) for g in rtamd.column_gens(g1, 60)]
    full = rtamd.runRender(env, gens[:48], ctx=gpu_ctx)
    assert len(full) == 24 and all(r.shape == (48, 3) for r in full)
    short = rtamd.runRender(env, gens[:41], ctx=gpu_ctx)
    assert all(r.shape == (41, 3) for r in short)
    assert all(np.array_equal(a, b[:41]) for a, b in zip(short, full))
    assert all(np.array_equal(a, b) for a, b in zip(rtamd.runRender(env, gens, ctx=gpu_ctx), full))
    assert all(r.shape == (0, 3) for r in rtamd.runRender(env, [], ctx=gpu_ctx))


@pytest.mark.parametrize("parts", [("fog2", "boxes", "light"), ("boxes", "light", "fog1")])
def test_grazing_rays_closest_hits(gpu_ctx, parts):
    """Rays lying in the face planes of the box field (the Lambertian quirk's +x light direction from a
    box top, nwf_parts.grazing_rays) over a world walked in the reference's order (media): exact ties
    between neighbouring faces, rect hits at t = NaN (rectHit does not reject a NaN t, Lib.hs:1014-1015)
    and boxes whose per-axis test fails on a NaN slab quotient (Lib.hs:798-814). The recursive walk
    must give the oracle's closest hits with the joint slab filter as with the reference's test: the
    joint filter's fast path drops a NaN bound (fmin / fmax), so a NaN closest hit sends it to the exact
    test. Medium hits: t within 8 ulps (OCML vs glibc log)."""
    from nwf_parts import grazing_rays, scene
    sc, _ = scene(list(parts))
    gpu_ctx.upload(sc)
    rays = grazing_rays(sc, 1 << 15, np.random.default_rng(3))
    ref = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    mats = sc.materials["type"]
    assert np.isnan(ref[:, 1]).sum() > 100  # (NaN-t hits occur)
    for flags in (0, rtamd.RT_FLAG_REFERENCE_CULL):
        got = gpu_ctx.closest_hits(rays, 1e-4, np.inf, seed=3, flags=flags)
        same = np.all((got == ref) | (np.isnan(got) & np.isnan(ref)), axis=1)
        med = (ref[:, 0] == 1) & (got[:, 11] == ref[:, 11]) & (mats[ref[:, 11].astype(int)] == 4)
        close = med & (np.abs(got[:, 1] - ref[:, 1]) <= 8 * np.spacing(np.abs(ref[:, 1])))
        print(f"{'+'.join(parts)} flags {flags}: {int((~same).sum())} rays differ, all medium t within 8 ulps: "
              f"{bool(np.all(same | close))}")
        assert np.all(same | close), f"{int((~(same | close)).sum())} rays differ"


def test_exact_trace_matches_oracle(gpu_ctx):
    """rt_debug_exact_trace against oracle_exact_trace: every path segment of a next_week_final column in
    tier A with RT_FLAG_SHARED_LIBM — scattered ray and generator state after each segment — bit for bit
    (the tool that localised the two round-5 tier-A divergences to one segment each)."""
    earth = np.load(_earth_path())["rgb"]
    sc, g1 = _scene("next_week_final", earth=earth)
    cam = rtamd.camera("next_week", 48, 48)
    gens = rtamd.column_gens(g1, 48)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(48, 48, 4, 50, rtamd.RT_RNG_EXACT, flags=rtamd.RT_FLAG_SHARED_LIBM)
    for col in (0, 17, 30):
        a = gpu_ctx.exact_trace(cam, p, gens, col)
        b = pyoracle.exact_trace(sc, cam, p, gens, col)
        assert len(a) == len(b) > 48 * 4
        assert np.array_equal(a, b, equal_nan=True), f"column {col}: first difference at record " \
            f"{int(np.argmax(~np.all((a == b) | (np.isnan(a) & np.isnan(b)), axis=1)))}"


@pytest.mark.parametrize("walk", [rtamd.RT_DEBUG_RESUMABLE, rtamd.RT_DEBUG_WIDE])
def test_nan_rays_hit_nothing(gpu_ctx, walk):
    """Rays with a NaN in the origin or direction (the segment after a rect hit at t = NaN, from the
    Lambertian quirk's +x ray along a box top) hit nothing, as in the reference, whose root box test fails
    for them: the 4-wide walk's fp32 test rejects every child (set_ray32) instead of accepting them all,
    which walked the whole tree per segment and let rect leaves take t = NaN. Checked against the oracle
    with ordinary rays mixed in, and on a tier-B render of the box field: per-sample work stays that of a
    culling walk (it was 745 4-wide nodes and 2200 leaf tests per sample)."""
    import nwf_parts
    sc, _ = nwf_parts.scene(["boxes"])
    gpu_ctx.upload(sc)
    rng = np.random.default_rng(5)
    n = 4096
    o = rng.uniform(-1000, 1000, (n, 3))
    o[:, 1] = rng.uniform(0, 300, n)
    d = rng.normal(0, 1, (n, 3))
    k = rng.integers(0, 6, n // 2)
    o[np.arange(n // 2)[k < 3], k[k < 3]] = np.nan
    d[np.arange(n // 2)[k >= 3], k[k >= 3] - 3] = np.nan
    rays = np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)
    got = gpu_ctx.closest_hits(rays, 1e-3, np.inf, seed=3, flags=walk)
    ref = pyoracle.closest_hits(sc, rays, 1e-3, np.inf, seed=3)
    assert not got[: n // 2, 0].any() and not ref[: n // 2, 0].any()
    assert got[n // 2:, 0].sum() > n // 8
    assert np.array_equal(got[:, [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]], ref[:, [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]])
    if walk == rtamd.RT_DEBUG_WIDE:
        cam = rtamd.camera("next_week", 96, 96)
        p = rtamd.make_params(96, 96, 8, 50, rtamd.RT_RNG_PHILOX, seed=1024)
        w = gpu_ctx.render_work(cam, p)
        per = {f: w[f] / w["samples"] for f in ("prim_tests", "wide_nodes")}
        print(f"box field, tier B 96x96x8: {per}")
        assert per["prim_tests"] < 20 and per["wide_nodes"] < 60


def test_nan_rays_take_no_hoisted_medium(gpu_ctx):
    """the tier-B walk prelude takes a world's hoisted media (RT_BVH_MEDIA_FIRST) without the
    chain's box tests. A ray with a NaN in its origin or direction (the segment after a rect hit at t = NaN)
    fails the reference's root box test (src/Lib.hs:798-814) and so never reaches a medium; with a cuboid
    boundary the boundary's t would be NaN, which the medium's range tests pass (a finite candidate). The
    debug walk runs the render loop's prelude (rt_debug_closest_hits, RT_DEBUG_RESUMABLE): a fog with a
    cuboid boundary over a 24-sphere world and a sky background, NaN rays and ordinary rays inside the fog,
    against the oracle (the reference's recursion over the caller's tree)."""
    b = rtamd.Builder(rtamd.randGen(7))
    lam = b.lambertian(b.constantColor(0.7, 0.6, 0.5))
    items = [b.sphere((3.0 * x, 1.0, 3.0 * z), 1.0, lam) for x in range(-3, 3) for z in range(-2, 2)]
    fog = b.constantMedium(0.05, b.constantColor(1.0, 1.0, 1.0), b.cuboid((-20.0, -1.0, -20.0), (20.0, 10.0, 20.0), lam))
    sc = b.finish(b.makeBVH((0.0, 1.0), items + [fog]), -1, (0.5, 0.7, 1.0))
    rb = rtamd.rebuilt_scene(sc)
    assert rb.nodes["c"][rb.desc.world_root] & rtamd.RT_BVH_MEDIA_FIRST  # (the fog is hoisted)
    gpu_ctx.upload(sc)
    rng = np.random.default_rng(11)
    n = 1 << 14
    o = rng.uniform(-15, 15, (n, 3))
    o[:, 1] = rng.uniform(0, 8, n)
    d = rng.normal(0, 1, (n, 3))
    k = rng.integers(0, 6, n // 2)
    o[np.arange(n // 2)[k < 3], k[k < 3]] = np.nan
    d[np.arange(n // 2)[k >= 3], k[k >= 3] - 3] = np.nan
    rays = np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)
    got = gpu_ctx.closest_hits(rays, 1e-4, np.inf, seed=3, flags=rtamd.RT_DEBUG_RESUMABLE)
    ref = pyoracle.closest_hits(sc, rays, 1e-4, np.inf, seed=3)
    assert not ref[: n // 2, 0].any() and not got[: n // 2, 0].any(), "a NaN ray took a hit"
    assert got[n // 2:, 0].sum() > n // 8
    mats = sc.materials["type"]
    # (sphere u, v go through atan / asin: OCML vs glibc, within 2e-15; every other field exact, or for a
    # medium hit its t through log within 8 ulps)
    ex = [0, 1, 2, 3, 4, 5, 6, 7, 10, 11]
    same = np.all((got[:, ex] == ref[:, ex]) | (np.isnan(got[:, ex]) & np.isnan(ref[:, ex])), axis=1)
    same &= np.all(np.abs(got[:, 8:10] - ref[:, 8:10]) <= 2e-15, axis=1)
    med = (ref[:, 0] == 1) & (got[:, 11] == ref[:, 11]) & (mats[ref[:, 11].astype(int)] == 4)
    close = med & (np.abs(got[:, 1] - ref[:, 1]) <= 8 * np.spacing(np.abs(ref[:, 1])))
    print(f"hoisted cuboid fog: {int(med.sum())} medium hits, {int((~same).sum())} rays not bit-identical "
          f"(medium t within 8 ulps: {bool(np.all(same | close))})")
    bad = ~(same | close)
    if bad.any():
        import os
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez("gpurun_out/hoisted_cuboid_fog.npz", rays=rays[bad], got=got[bad], ref=ref[bad])
    assert not bad.any(), f"{int(bad.sum())} rays differ"


def test_quantised_tree_renders_the_same_image(gpu_ctx, monkeypatch):
    """RTAMD_QNODE=1 (A/B: the global-memory spheres kernel over the quantised 64-byte nodes and the
    32-byte sphere leaves) renders the default build's image, bytes and linear averages."""
    sc, _ = _scene("stress_spheres", param=3000)
    cam = rtamd.camera("random_scene", 96, 64)
    p = rtamd.make_params(96, 64, 4, 50, rtamd.RT_RNG_PHILOX, seed=9)
    monkeypatch.setenv("RTAMD_LDS", "0")  # (the global-memory kernel in both runs)
    gpu_ctx.upload(sc)
    rgb0, lin0, _ = gpu_ctx.render(cam, p, linear=True)
    monkeypatch.setenv("RTAMD_QNODE", "1")
    gpu_ctx.upload(sc)
    rgb1, lin1, _ = gpu_ctx.render(cam, p, linear=True)
    assert gpu_ctx.last_launch()["loop"] == 2
    assert np.array_equal(rgb0, rgb1)
    assert np.array_equal(np.isnan(lin0), np.isnan(lin1)) and np.array_equal(lin0[~np.isnan(lin0)], lin1[~np.isnan(lin1)])


@pytest.mark.parametrize("name,cam", [("next_week_final", "next_week"), ("cornell_smoke", "cornell")])
def test_tail_units_do_not_change_the_image(gpu_ctx, name, cam, monkeypatch):
    """The full variants' replacement loop deals the last work-items of a launch one sample per unit
    (RTAMD_TAIL), their colours summed afterwards in sample order (tail_combine), as the lane that renders
    a whole chunk sums them: the image and the linear averages are identical with no tail, the default
    tail, every item in the tail, and every item in the tail with the chunks rendered in batches. At
    128x96x704 a chunk holds 8 samples (rt_sample_chunk), so tail units are single samples of 8-sample
    chunks; every sample is rendered once (the counting build's count)."""
    earth = np.load(_earth_path())["rgb"] if name == "next_week_final" else None
    sc, _ = _scene(name, earth=earth)
    c = rtamd.camera(cam, 128, 96)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(128, 96, 704, 50, rtamd.RT_RNG_PHILOX, seed=23)
    slab_chunk = 128 * 96 * 3 * 8
    out = []
    for tail, cap in (("0", 0), (None, 0), ("65536", 0), ("65536", 7 * slab_chunk)):
        if tail is None:
            monkeypatch.delenv("RTAMD_TAIL", raising=False)
        else:
            monkeypatch.setenv("RTAMD_TAIL", tail)
        if cap:
            monkeypatch.setenv("RTAMD_PARTIAL_CAP", str(cap))
        else:
            monkeypatch.delenv("RTAMD_PARTIAL_CAP", raising=False)
        out.append(gpu_ctx.render(c, p, linear=True))
        info = gpu_ctx.last_launch()
        assert info["loop"] == 1 and info["chunk"] == 8 and info["chunk_batches"] == (13 if cap else 1)
        assert gpu_ctx.render_work(c, p)["samples"] == 128 * 96 * 704
    for rgb, lin, _ in out[1:]:
        assert np.array_equal(rgb, out[0][0]) and np.array_equal(lin, out[0][1], equal_nan=True)

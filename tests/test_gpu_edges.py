"""GPU edge cases of the render boundary against the oracle: degenerate and ragged image sizes,
one sample, depth 0 and 1 (rayColor's `d <= 0 -> black`, src/Lib.hs:1298-1300), an empty world
(Unhittable, background only), a world that is a single primitive (no BVH), lights that are a
single primitive, camera rays from inside a sphere, and shard counts that leave shards without
tiles. Tier B unless stated; the same tolerance as tests/test_gpu_parity.py."""
import numpy as np
import pytest

import pyoracle
import rtamd
from conftest import parity

pytestmark = pytest.mark.gpu


def _cmp(ctx, scene, cam, p, col_gens=None):
    ctx.upload(scene)
    rgb_g, lin_g, gens_g = ctx.render(cam, p, col_gens, linear=True, want_gens=col_gens is not None)
    rgb_o, lin_o, gens_o, _ = pyoracle.render(scene, cam, p, col_gens=col_gens)
    ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
    print(f"{p.width}x{p.height}x{p.spp} d{p.max_depth}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, "
          f"max |d| {dmax:.3g}")
    assert ok >= 0.999 and eq >= 0.999, (ok, eq, dmax)
    if col_gens is not None:
        assert np.array_equal(gens_g, gens_o)
    return rgb_g, lin_g


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (17, 13), (8, 40), (129, 1)])
def test_ragged_and_tiny_images(gpu_ctx, w, h):
    """Image sizes that are not multiples of the 16-pixel tile or the 8x8 block (padding work-items
    fall outside the image and are never stored)."""
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", w, h)
    _cmp(gpu_ctx, sc, cam, rtamd.make_params(w, h, 3, 20, rtamd.RT_RNG_PHILOX, seed=31))


@pytest.mark.parametrize("rng", [rtamd.RT_RNG_PHILOX, rtamd.RT_RNG_EXACT])
@pytest.mark.parametrize("depth", [0, 1])
def test_depth_zero_and_one(gpu_ctx, depth, rng):
    """maxDepth 0: every sample is black (rayColor returns 0 before tracing, Lib.hs:1298-1300);
    depth 1: one segment, then black unless the first hit emits or misses."""
    sc, g1 = rtamd.make_scene("cornell", rtamd.randGen(1024))
    cam = rtamd.camera("cornell", 24, 24)
    gens = rtamd.column_gens(g1, 24) if rng == rtamd.RT_RNG_EXACT else None
    rgb, lin = _cmp(gpu_ctx, sc, cam, rtamd.make_params(24, 24, 4, depth, rng, seed=3), col_gens=gens)
    if depth == 0:
        assert not rgb.any() and not lin.any()


def test_one_sample(gpu_ctx):
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 64, 40)
    _cmp(gpu_ctx, sc, cam, rtamd.make_params(64, 40, 1, 50, rtamd.RT_RNG_PHILOX, seed=5))


def test_empty_world_is_background(gpu_ctx):
    """World = Unhittable (Lib.hs:584): every ray misses, every pixel is the background."""
    b = rtamd.Builder(rtamd.randGen(1))
    world = b.unhittable()
    sc = b.finish(world, -1, (0.25, 0.5, 1.0))
    cam = rtamd.camera("random_scene", 32, 16)
    rgb, lin = _cmp(gpu_ctx, sc, cam, rtamd.make_params(32, 16, 2, 10, rtamd.RT_RNG_PHILOX, seed=1))
    assert np.allclose(lin, [0.25, 0.5, 1.0])
    assert np.all(rgb == rgb[0, 0])


def test_single_primitive_world_and_light(gpu_ctx):
    """A world that is one sphere (no BVH node at all) lit through a lights tree that is one XZ
    rect (htblRandom / htblPdfValue of a bare Rect, Lib.hs:673-724), camera inside the sphere."""
    b = rtamd.Builder(rtamd.randGen(9))
    white = b.lambertian(b.constantColor(0.73, 0.73, 0.73))
    light = b.diffuseLight(b.constantColor(15, 15, 15))
    shell = b.sphere((0.0, 0.0, 0.0), 50.0, white)
    lamp = b.rect(rtamd.XZPlane, -5, 5, -5, 5, 49.0, light)
    world = b.makeBVH((0.0, 1.0), [shell, lamp])
    sc = b.finish(world, lamp, (0.0, 0.0, 0.0))
    cam = rtamd.newCamera((0.0, 0.0, -20.0), (0.0, 10.0, 0.0), (0.0, 1.0, 0.0), 70.0, 1.0, 0.0, 10.0, 0.0, 1.0)
    rgb, _ = _cmp(gpu_ctx, sc, cam, rtamd.make_params(40, 40, 6, 20, rtamd.RT_RNG_PHILOX, seed=8))
    assert rgb.any()
    b2 = rtamd.Builder(rtamd.randGen(9))
    m2 = b2.lambertian(b2.constantColor(0.5, 0.6, 0.7))
    only = b2.sphere((0.0, 0.0, 0.0), 3.0, m2)
    sc2 = b2.finish(only, -1, (0.7, 0.8, 0.9))
    cam2 = rtamd.camera("random_scene", 40, 30)
    _cmp(gpu_ctx, sc2, cam2, rtamd.make_params(40, 30, 4, 10, rtamd.RT_RNG_PHILOX, seed=2))


def test_more_shards_than_tiles(gpu_ctx):
    """A 20x20 image has 4 tiles of 16: with 6 shards two of them own no tile (their slabs are all
    padding); the assembled image still equals the one-shard render."""
    import torch
    sc, _ = rtamd.make_scene("three_spheres", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 20, 20)
    gpu_ctx.upload(sc)
    base = rtamd.make_params(20, 20, 4, 10, rtamd.RT_RNG_PHILOX, seed=4, tile=16)
    ref, _, _ = gpu_ctx.render(cam, base)
    shards = 6
    _, _, slab = rtamd.shard_geometry(rtamd.make_params(20, 20, 4, 10, shard_count=shards, tile=16))
    slabs = torch.zeros((shards, slab, 3), dtype=torch.uint8, device="cuda")
    for r in range(shards):
        p = rtamd.make_params(20, 20, 4, 10, rtamd.RT_RNG_PHILOX, seed=4, shard_rank=r, shard_count=shards, tile=16)
        gpu_ctx.render_shard_async(cam, p, slabs[r].data_ptr())
    torch.cuda.synchronize()
    img = torch.zeros((20, 20, 3), dtype=torch.uint8, device="cuda")
    gpu_ctx.assemble_async(rtamd.make_params(20, 20, 4, 10, shard_count=shards, tile=16), slabs.data_ptr(), img.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy(), ref)

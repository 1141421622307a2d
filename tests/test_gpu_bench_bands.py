"""Parity at the bench launches: every bench frame (bench.py CONFIGS c2..c5, SURVEY.md
8d) is rendered whole on the device through the path bench.py times — rtamd.frame.ShardedFrame:
rt_render_shard_async into a tile slab, rt_assemble_async into the image, same kernel instantiation,
chunking (rt_sample_chunk of the full frame) and work decomposition — and a full-width band of rows
is compared with the oracle's render of the same rows of the same frame (tests/golden/bench_bands.npz,
made by tests/golden/make_band_goldens.py; app/Main.hs:50-62 renders whole frames the same way).

Tolerance (north star / SURVEY.md 8d): |d| <= 1e-3 per channel on the displayed float
sqrt(clamp(0, 0.999)(avg)), NaN == NaN, for >= 99.9 % of channels, and >= 99.9 % equal bytes; the
NaN mask must match exactly. Each test prints the observed fractions and max |d|.

The bench frames are mostly NaN under the reference's Lambertian light-mixture quirk (C2's band
99.9 %, C4's 100 % of channels): the *z bands render the same launches with RT_FLAG_NAN_ZERO (a NaN
sample channel adds 0, on both sides), so that every sample's finite colour is compared.
"""
import os

import numpy as np
import pytest

import rtamd
from conftest import parity

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
B = np.load(os.path.join(HERE, "golden", "bench_bands.npz"))
SCENES = {  # key -> (scene, camera, param, earth), as bench.py CONFIGS
    "c2": ("random_book_one", "random_scene", 0, False),
    "c3": ("cornell", "cornell", 0, False),
    "c4": ("next_week_final", "next_week", 0, True),
    "c5": ("stress_spheres", "random_scene", 100000, False),
}
_scene_cache = {}


def _scene(cfg):
    if cfg not in _scene_cache:
        name, _, param, earth = SCENES[cfg]
        e = np.load(os.path.join(HERE, "golden", "earthmap_rgb8.npz"))["rgb"] if earth else None
        _scene_cache.clear()  # (one big scene at a time: C5 holds 100k spheres)
        _scene_cache[cfg] = rtamd.make_scene(name, rtamd.randGen(1024), param=param, earth=e)[0]
    return _scene_cache[cfg]


def render_like_bench(ctx, cfg, W, H, spp, depth, seed, flags):
    """One bench step at N = 1 (ShardedFrame, as bench.py), plus the linear slab assembled the same way."""
    import torch
    from rtamd.frame import ShardedFrame, device_assembler, device_renderer
    sc = _scene(cfg)
    cam = rtamd.camera(SCENES[cfg][1], W, H)
    ctx.upload(sc)
    p = rtamd.make_params(W, H, spp, depth, rtamd.RT_RNG_PHILOX, seed=seed, flags=flags)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    lin_slab = torch.zeros((rtamd.shard_geometry(p)[2], 3), dtype=torch.float64, device=dev)

    def render(params, slab):  # the bench renderer, with the optional linear slab filled too
        ctx.render_shard_async(cam, params, slab.data_ptr(), lin_slab.data_ptr(), st)

    frame = ShardedFrame(p, 1, 0, dev, render=render, assemble=device_assembler(ctx, st))
    frame.step(kernel_ms=ctx.last_kernel_ms)
    lin = torch.zeros((H, W, 3), dtype=torch.float64, device=dev)
    ctx.assemble_linear_async(p, lin_slab.data_ptr(), lin.data_ptr(), st)
    torch.cuda.synchronize()
    t = frame.finish()[0]
    del device_renderer
    return frame.image.cpu().numpy(), lin.cpu().numpy(), t["kernel_ms"], ctx.last_launch()


@pytest.mark.parametrize("key", ["c2", "c3", "c4", "c5", "c5b", "c4s", "c2z", "c4z", "c5z", "c5bz"])
def test_bench_frame_band_matches_oracle(gpu_ctx, key):
    W, H, spp, depth, seed, r0, flags = [int(x) for x in B[f"{key}_frame"]]
    rgb_o, lin_o = B[f"{key}_rgb"], B[f"{key}_lin"]
    rows = rgb_o.shape[0]
    rgb, lin, kms, launch = render_like_bench(gpu_ctx, key[:2], W, H, spp, depth, seed, flags)
    band_rgb, band_lin = rgb[r0:r0 + rows], lin[r0:r0 + rows]
    ok, eq, dmax = parity(band_lin, lin_o, band_rgb, rgb_o)
    nan_g, nan_o = np.isnan(band_lin), np.isnan(lin_o)
    print(f"{key}: {W}x{H}x{spp} rows {r0}..{r0 + rows - 1}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, "
          f"max |d| {dmax:.3g}, NaN channels {nan_o.mean():.4f}, kernel {kms:.1f} ms, launch {launch}")
    if key.startswith("c5"):  # the 100k-sphere tree does not fit LDS: the global-memory 4-wide kernel
        assert launch["loop"] == 2 and not launch["lds_staged"] and launch["variant"] == 256 and launch["waves"] == 3
    if key.startswith("c4"):  # media + frames: the replacement loop's mixed walk over 4-wide subtrees
        assert launch["loop"] == 1 and launch["variant"] & 1024 and launch["wide_nodes"] > 0
    # the bench frames' own chunking (rt_sample_chunk): 8-sample chunks at 500 / 1000 spp, 16 at C5's 2000
    # spp, whose 125 chunks' sums (24.9 GB) are rendered in batches of at most 2 GiB of chunk sums
    assert launch["chunk"] == {500: 8, 1000: 8, 2000: 16, 16: 8, 4: 4}[spp]
    if key.startswith("c5b"):
        assert launch["chunk_batches"] == 13
    print(f"{key}: NaN masks differ in {int((nan_g != nan_o).sum())} channels")
    assert (nan_g == nan_o).all(), f"{key}: NaN masks differ"  # (NaN comes from pdf 0, never from rounding)
    assert ok >= 0.999, f"{key}: only {ok:.5f} of channels within 1e-3 (max |d| {dmax:.3g})"
    assert eq >= 0.999, f"{key}: only {eq:.5f} of bytes equal"
    if flags & rtamd.RT_FLAG_NAN_ZERO:
        assert not nan_o.any()

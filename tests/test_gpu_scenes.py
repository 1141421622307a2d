"""GPU: scenes built through the reference's constructor API (rtamd.Builder, the src/Lib.hs
surface) that exercise the device path's structural limits — instance frames nested within and
beyond RT_MAX_FRAMES (replacement loop vs per-sample loop), media inside frames — and the
upload's validation of malformed descriptors (error codes, no fallback)."""
import ctypes as C
import os

import numpy as np
import pytest

import pyoracle
import rtamd
from conftest import parity

pytestmark = pytest.mark.gpu


def _frames_scene(depth, medium=False):
    """Ground + a BVH of small spheres wrapped in `depth` alternating Translate/Rotate frames
    (Lib.hs:561-576) + optionally a ConstantMedium inside the frames, all under makeBVH."""
    b = rtamd.Builder(rtamd.randGen(77))
    white = b.lambertian(b.constantColor(0.73, 0.73, 0.73))
    red = b.lambertian(b.constantColor(0.65, 0.05, 0.05))
    glass = b.dielectric(1.5)
    metal = b.metal(b.constantColor(0.8, 0.8, 0.9), 0.1)
    rng = np.random.default_rng(3)
    items = []
    for i in range(24):
        c = (float(rng.uniform(-2, 2)), float(rng.uniform(0.2, 2)), float(rng.uniform(-2, 2)))
        items.append(b.sphere(c, float(rng.uniform(0.1, 0.4)), [white, red, glass, metal][i % 4]))
    if medium:
        boundary = b.sphere((0.0, 1.0, 0.0), 0.8, glass)
        items.append(b.constantMedium(0.6, b.constantColor(0.2, 0.4, 0.9), boundary))
    inner = b.makeBVH((0.0, 1.0), items)
    for k in range(depth):
        inner = b.translate((0.3, 0.0, -0.2), inner) if k % 2 == 0 else b.rotate(rtamd.YAxis, 17.0, inner)
    ground = b.sphere((0.0, -1000.0, 0.0), 1000.0, white)
    world = b.makeBVH((0.0, 1.0), [ground, inner])
    return b.finish(world, -1, (0.7, 0.8, 1.0))


@pytest.mark.parametrize("depth,medium", [(2, False), (2, True), (6, False)])
def test_nested_frames(gpu_ctx, depth, medium, monkeypatch):
    """Frames nested 2 deep (replacement loop, Side slots) and 6 deep (> RT_MAX_FRAMES: per-sample
    loop), with a medium inside the frames: the oracle's image within the tolerance, and the two
    loops byte-identical where both apply."""
    sc = _frames_scene(depth, medium)
    cam = rtamd.camera("random_scene", 64, 40)
    p = rtamd.make_params(64, 40, 6, 20, rtamd.RT_RNG_PHILOX, seed=9)
    gpu_ctx.upload(sc)
    rgb, lin, _ = gpu_ctx.render(cam, p, linear=True)
    rgb_o, lin_o, _, _ = pyoracle.render(sc, cam, p)
    ok, eq, dmax = parity(lin, lin_o, rgb, rgb_o)
    print(f"frames depth {depth} medium {medium}: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, max |d| {dmax:.3g}")
    assert ok >= 0.999 and eq >= 0.999, (ok, eq, dmax)
    monkeypatch.setenv("RTAMD_REPLACE", "0")
    rgb_s, lin_s, _ = gpu_ctx.render(cam, p, linear=True)
    assert np.array_equal(rgb, rgb_s) and np.array_equal(lin, lin_s, equal_nan=True)


def _desc_with_nodes(sc, nodes, **over):
    """A copy of scene `sc`'s descriptor pointing at `nodes` (kept alive by the caller)."""
    d = rtamd.rt_scene_desc()
    C.pointer(d)[0] = sc.desc
    d.nodes = nodes.ctypes.data_as(C.POINTER(rtamd.rt_node))
    d.n_nodes = len(nodes)
    for k, v in over.items():
        setattr(d, k, v)
    return d


def _upload_raw(ctx, d):
    return rtamd.lib().rt_upload_scene(ctx._h, C.byref(d))


def test_upload_rejects_malformed_scenes(gpu_ctx):
    """rt_upload_scene validates the DAG and its references: RT_E_INVALID for a child that does not
    precede its parent, a material or root out of range; RT_E_UNSUPPORTED for a medium in the
    lights tree. A rejected upload leaves the previously uploaded scene in place, untouched."""
    sc, _ = rtamd.make_scene("cornell", rtamd.randGen(1024))
    cam = rtamd.camera("cornell", 16, 16)
    p = rtamd.make_params(16, 16, 2, 10, rtamd.RT_RNG_PHILOX, seed=4)
    gpu_ctx.upload(sc)
    before, _, _ = gpu_ctx.render(cam, p)
    base = np.array(sc.nodes, copy=True)
    bvh = np.where(base["type"] == rtamd.RT_NODE_BVH)[0][0]
    bad = base.copy()
    bad["a"][bvh] = len(bad) - 1 if len(bad) - 1 > bvh else bvh  # child at or after its parent
    assert _upload_raw(gpu_ctx, _desc_with_nodes(sc, bad)) == rtamd.RT_E_INVALID
    assert b"precede" in rtamd.lib().rt_last_error()
    bad = base.copy()
    sph = np.where(np.isin(base["type"], [rtamd.RT_NODE_RECT_XZ, rtamd.RT_NODE_SPHERE]))[0][0]
    bad["a"][sph] = 10_000  # material out of range
    assert _upload_raw(gpu_ctx, _desc_with_nodes(sc, bad)) == rtamd.RT_E_INVALID
    assert _upload_raw(gpu_ctx, _desc_with_nodes(sc, base, world_root=len(base) + 5)) == rtamd.RT_E_INVALID
    smoke, _ = rtamd.make_scene("cornell_smoke", rtamd.randGen(1024))
    snodes = np.array(smoke.nodes, copy=True)
    medium = int(np.where(snodes["type"] == rtamd.RT_NODE_CONSTANT_MEDIUM)[0][0])
    rc = _upload_raw(gpu_ctx, _desc_with_nodes(smoke, snodes, lights_root=medium))
    assert rc == rtamd.RT_E_UNSUPPORTED, rc
    after, _, _ = gpu_ctx.render(cam, p)
    assert np.array_equal(before, after)


def test_upload_rejects_null_image_pool_and_keeps_scene(gpu_ctx):
    """image_pool_bytes > 0 with a null pool is refused (the device would read textures through a
    null pointer); the previously uploaded scene stays usable."""
    import ctypes as C
    sc, _ = rtamd.make_scene("three_spheres", rtamd.randGen(1024))
    gpu_ctx.upload(sc)
    cam = rtamd.camera("random_scene", 32, 16)
    p = rtamd.make_params(32, 16, 2, 5, rtamd.RT_RNG_PHILOX, seed=1)
    before, _, _ = gpu_ctx.render(cam, p)
    earth = np.load(os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz"))["rgb"]
    bad, _ = rtamd.make_scene("earth", rtamd.randGen(1024), earth=earth)
    d = rtamd.rt_scene_desc()
    C.pointer(d)[0] = bad.desc
    d.image_pool = C.POINTER(C.c_uint8)()
    rc = rtamd.lib().rt_upload_scene(gpu_ctx._h, C.byref(d))
    assert rc == rtamd.RT_E_INVALID and b"image_pool" in rtamd.lib().rt_last_error()
    after, _, _ = gpu_ctx.render(cam, p)
    assert np.array_equal(before, after)


def test_launches_on_two_streams_are_ordered(gpu_ctx):
    """Shard launches on two different streams share the ctx's work counter and chunk-sum buffer:
    the second waits for the first, so both slabs equal their one-stream renders."""
    import torch
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    gpu_ctx.upload(sc)
    cam = rtamd.camera("random_scene", 96, 64)
    ps = [rtamd.make_params(96, 64, 40, 20, rtamd.RT_RNG_PHILOX, seed=s, shard_rank=0, shard_count=1) for s in (3, 4)]
    _, _, slab = rtamd.shard_geometry(ps[0])
    ref = []
    for p in ps:
        buf = torch.zeros((slab, 3), dtype=torch.uint8, device="cuda")
        gpu_ctx.render_shard_async(cam, p, buf.data_ptr())
        torch.cuda.synchronize()
        ref.append(buf.cpu().numpy())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [torch.zeros((slab, 3), dtype=torch.uint8, device="cuda") for _ in ps]
    for p, b, st in zip(ps, bufs, streams):
        gpu_ctx.render_shard_async(cam, p, b.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    for b, r in zip(bufs, ref):
        assert np.array_equal(b.cpu().numpy(), r)


@pytest.mark.parametrize("name,camname", [("next_week_final", "next_week"), ("random", "random_scene")])
def test_rebuilt_world_uploaded_again(gpu_ctx, name, camname):
    """A caller's world tree that already holds RT_BVH_ORDERED nodes (rt_rebuild_bvh output, e.g.
    rtamd.rebuilt_scene, uploaded again): media and textured worlds render to the oracle's image of
    the original scene (next_week_final: media, frames, Perlin and image textures; random: moving
    spheres, checker and image textures), and walks redone for an exact tie treat every node with the reference's
    semantics (before, such a redo could flag the same tie forever)."""
    earth = np.load(os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz"))["rgb"]
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024), earth=earth)
    rb = rtamd.rebuilt_scene(sc)
    assert (rb.nodes["c"] & rtamd.RT_BVH_ORDERED).any()
    cam = rtamd.camera(camname, 48, 40)
    p = rtamd.make_params(48, 40, 4, 50, rtamd.RT_RNG_PHILOX, seed=13)
    gpu_ctx.upload(rb)
    rgb, lin, _ = gpu_ctx.render(cam, p, linear=True)
    w = gpu_ctx.render_work(cam, p)
    rgb_o, lin_o, _, _ = pyoracle.render(sc, cam, p)
    ok, eq, dmax = parity(lin, lin_o, rgb, rgb_o)
    print(f"{name} rebuilt + re-uploaded: channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, max |d| {dmax:.3g}, "
          f"tie redos {w['tie_redos']}")
    assert w["samples"] == 48 * 40 * 4
    assert ok >= 0.999 and eq >= 0.999, (ok, eq, dmax)


def _coplanar_scene(kind):
    """Two overlapping XY rects in the plane z = 0 (every ray through the overlap hits both at the same t)
    in front of 20 small spheres (enough leaves for the SAH rebuild, whose walk detects exact ties):
    kind "same" = one material with a constant texture (records shade identically: no redo, tie_same),
    "diff" = two materials (redo in the reference's order), "uv" = one material with an image texture
    (u, v are read: redo)."""
    b = rtamd.Builder(rtamd.randGen(5))
    if kind == "uv":
        img = np.arange(16 * 8 * 3, dtype=np.uint8).reshape(8, 16, 3) * 5
        ma = mb = b.lambertian(b.imageTexture(img))
    else:
        ma = b.lambertian(b.constantColor(0.8, 0.3, 0.2))
        mb = ma if kind == "same" else b.metal(b.constantColor(0.2, 0.7, 0.9), 0.3)
    items = [b.rect(rtamd.XYPlane, -1.0, 1.0, -1.0, 1.0, 0.0, ma), b.rect(rtamd.XYPlane, -0.5, 1.5, -1.2, 0.8, 0.0, mb)]
    rng = np.random.default_rng(9)
    grey = b.lambertian(b.constantColor(0.5, 0.5, 0.5))
    for _ in range(20):
        items.append(b.sphere((float(rng.uniform(-3, 3)), float(rng.uniform(-3, 3)), float(rng.uniform(-6, -2))), 0.3,
                              grey))
    return b.finish(b.makeBVH((0.0, 1.0), items), -1, (0.7, 0.8, 1.0))


@pytest.mark.parametrize("kind", ["same", "diff", "uv"])
def test_coplanar_ties(gpu_ctx, kind):
    """tie_same (rt_trace.h): an exact tie between two rect faces on one plane orientation needs no redo
    only when both records shade identically (same material, no (u, v)-reading texture); a different
    material or an image texture is redone in the reference's order. The counting build's tie-redo count
    says which happened; the image matches the oracle either way."""
    sc = _coplanar_scene(kind)
    info = rtamd.prepare_scene(sc)
    assert info["rebuilt_bvh"], info
    gpu_ctx.upload(sc)
    cam = rtamd.newCamera((0.3, 0.1, 4.0), (0.2, 0.0, 0.0), (0.0, 1.0, 0.0), 35.0, 1.0, 0.0, 4.0, 0.0, 1.0)
    # (depth 1: camera rays only — the Lambertian quirk's +x rays, with lights Unhittable, run in the
    # rects' plane and end on NaN-t hits, redone for their own reason, trav_take)
    p = rtamd.make_params(64, 64, 4, 1, rtamd.RT_RNG_PHILOX, seed=13)
    redos = gpu_ctx.render_work(cam, p)["tie_redos"]
    rgb_g, lin_g, _ = gpu_ctx.render(cam, p, linear=True)
    rgb_o, lin_o, _, _ = pyoracle.render(sc, cam, p)
    ok, eq, dmax = parity(lin_g, lin_o, rgb_g, rgb_o)
    print(f"coplanar {kind}: tie redos {redos}, channels within 1e-3 {ok:.6f}, bytes equal {eq:.6f}, max |d| {dmax:.3g}")
    assert ok >= 0.999 and eq >= 0.999
    if kind == "same":
        assert redos == 0
    else:
        assert redos > 100  # (the camera rays through the overlap)


@pytest.mark.parametrize("scene,camera,kinds", [
    ("random_book_one", "random_scene", {"wide", "leaf", "box+wide"}),   # the 4-wide walk (round 6)
    ("next_week_final", "next_week", None),                              # the mixed walk
])
def test_step_profile_bins(gpu_ctx, scene, camera, kinds):
    """rt_render_step_profile (scripts/step_profile.py): every walk reports its
    steps by kind with positive times. The 4-wide walk's steps are node steps, leaf steps, or node steps
    with a tie redo on the caller's tree; the mixed walk of next_week_final has steps at instance frames."""
    earth = np.load(os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz"))["rgb"]
    sc, _ = rtamd.make_scene(scene, rtamd.randGen(1024), earth=earth if scene == "next_week_final" else None)
    gpu_ctx.upload(sc)
    cam = rtamd.camera(camera, 64, 48)
    prof = gpu_ctx.step_profile(cam, rtamd.make_params(64, 48, 4, 50, rtamd.RT_RNG_PHILOX, seed=1024))
    print(f"{scene} step profile: {prof}")
    assert prof and all(ticks > 0 and n > 0 for ticks, n in prof.values())
    if kinds is not None:
        assert set(prof) <= kinds and {"wide", "leaf"} <= set(prof)
    else:
        assert any("frame" in k for k in prof) and any("wide" in k for k in prof)


def test_w8_tree_renders_the_same_image(gpu_ctx, monkeypatch):
    """The 8-wide tree as 4-wide record pairs (RTAMD_W8=1 at upload, F_W8 kernels; measured slower, A/B
    only: DESIGN.md §3.2e) renders the 4-wide tree's image bit for bit: the closest hit does not depend on
    the tree, exact ties aside, which both redo on the caller's tree."""
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 96, 64)
    p = rtamd.make_params(96, 64, 8, 50, rtamd.RT_RNG_PHILOX, seed=1024)
    gpu_ctx.upload(sc)
    rgb_a, lin_a, _ = gpu_ctx.render(cam, p, linear=True)
    monkeypatch.setenv("RTAMD_W8", "1")
    info = rtamd.prepare_scene(sc)
    gpu_ctx.upload(sc)
    rgb_b, lin_b, _ = gpu_ctx.render(cam, p, linear=True)
    launch = gpu_ctx.last_launch()
    print(f"w8: {info['n_wide_nodes']} records, stack bound {info['wide_stack_need']}, launch {launch}")
    assert launch["variant"] & 16384 and not launch["lds_staged"]  # (F_W8, from global memory)
    assert np.array_equal(rgb_a, rgb_b) and np.array_equal(lin_a, lin_b, equal_nan=True)

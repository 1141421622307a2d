"""Scene construction (CPU): the product's C++ builders (rtamd -> librtamd.so) against the
independent Python restatement (oracle/scenes_ref.py), structurally and bit for bit, including
the generator handed back after construction (g1, app/Main.hs:41,49)."""
import math
import os

import numpy as np
import pytest

import rtamd
import scenes_ref

EARTH = os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz")


def _earth():
    return np.load(EARTH)["rgb"]


@pytest.mark.parametrize("name", ["three_spheres", "random_book_one", "cornell", "cornell_smoke", "simple_light",
                                  "two_perlin_spheres", "two_spheres", "earth", "random", "next_week_final"])
@pytest.mark.parametrize("seed", [1024, 7])
def test_builder_matches_restatement(name, seed):
    earth = _earth() if name in ("earth", "random", "next_week_final") else None
    gen = rtamd.randGen(seed)
    scene, g1 = rtamd.make_scene(name, gen, earth=earth)
    w, l, bg, g1_ref = scenes_ref.build(name, gen, earth)
    assert g1 == g1_ref, "generator after construction differs"
    assert scenes_ref.canon_desc(scene) == scenes_ref.canon(w)
    lights = scene.desc.lights_root
    if l["kind"] == "unhittable":
        assert lights == -1
    else:
        assert scenes_ref.canon_desc(scene, lights) == scenes_ref.canon(l)
    assert tuple(scene.desc.background) == tuple(float(x) for x in bg)


def test_book_one_shape():
    """makeRandomSceneBookOne: 4 fixed + <= 484 random spheres, BVH sizes consistent."""
    scene, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    nodes = scene.nodes
    spheres = int((nodes["type"] == rtamd.RT_NODE_SPHERE).sum())
    assert 4 < spheres <= 488
    root = nodes[scene.desc.world_root]
    assert root["type"] == rtamd.RT_NODE_BVH and root["c"] == spheres


def test_single_item_bvh_duplicates_leaf():
    """makeBVH of one item builds BVHNode h h with size 1 (src/Lib.hs:948)."""
    b = rtamd.Builder(rtamd.randGen(3))
    m = b.lambertian(b.constantColor(0.5, 0.5, 0.5))
    s = b.sphere((0, 0, 0), 1.0, m)
    n = b.makeBVH((0.0, 1.0), [s])
    sc = b.finish(n, -1, (0, 0, 0))
    node = sc.nodes[n]
    assert node["a"] == node["b"] == s and node["c"] == 1


def test_bvh_consumes_one_draw_per_call():
    gen = rtamd.randGen(99)
    b = rtamd.Builder(gen)
    m = b.lambertian(b.constantColor(0.5, 0.5, 0.5))
    items = [b.sphere((i, 0, 0), 0.5, m) for i in range(5)]
    b.makeBVH(None, items)
    # 5 items -> calls: 5, 2, 3, 1, 2  => 5 draws
    g = scenes_ref.Gen(gen)
    for _ in range(5):
        g.D()
    assert b.gen == g.state


def test_unhittable_in_bvh_is_rejected():
    b = rtamd.Builder(rtamd.randGen(1))
    u = b.unhittable()
    with pytest.raises(rtamd.RTError):
        b.makeBVH(None, [u, u, u])


def test_bad_ids_are_rejected():
    b = rtamd.Builder(rtamd.randGen(1))
    with pytest.raises(rtamd.RTError):
        b.sphere((0, 0, 0), 1.0, 17)
    with pytest.raises(rtamd.RTError):
        b.translate((0, 0, 0), 5)
    with pytest.raises(rtamd.RTError):
        b.rect(7, 0, 1, 0, 1, 0, 0)


@pytest.mark.parametrize("name,w,h", [("cornell", 500, 500), ("random_scene", 1200, 800), ("two_spheres", 40, 40),
                                      ("next_week", 800, 800)])
def test_cameras_match_restatement(name, w, h):
    cam = rtamd.camera(name, w, h)
    args = {"cornell": ((278, 278, -800), (278, 278, 0.0), 40.0, 0.0, 10.0),
            "random_scene": ((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), 20.0, 0.1, 10.0),
            "two_spheres": ((26.0, 4.0, 6.0), (0.0, 2.0, 0.0), 20.0, 0.1, 20.0),
            "next_week": ((575, 278, -525), (320, 278, 0.0), 40.0, 0.1, 580.0)}[name]
    lf, la, vfov, ap, fd = args
    ref = scenes_ref.new_camera(lf, la, (0.0, 1.0, 0.0), vfov, w / h, ap, fd, 0.0, 1.0)
    for k in ("origin", "llc", "horiz", "vert", "u", "v", "w"):
        assert tuple(getattr(cam, k)) == tuple(float(x) for x in ref[k]), k
    assert cam.lens_radius == ref["lens_radius"]


def test_rotate_box_uses_extrapolated_corners():
    """rotate's fold visits i,j,k in {0,1,2} (src/Lib.hs:761): the box is larger than the exact one."""
    b = rtamd.Builder(rtamd.randGen(1))
    m = b.lambertian(b.constantColor(0.5, 0.5, 0.5))
    c = b.cuboid((0, 0, 0), (1, 1, 1), m)
    r = b.rotate(1, 0.0, c)  # zero angle: exact box would be [0,1]^3
    top = b.makeBVH(None, [r, r])
    sc = b.finish(top, -1, (0, 0, 0))
    f = sc.nodes[top]["f"]
    assert f[3] == 2.0 and f[0] == 0.0  # i = 2 extrapolates to 2*max - min


def test_perlin_tables_are_permutations():
    b = rtamd.Builder(rtamd.randGen(5))
    t = b.makePerlin(1.0)
    sc = b.finish(b.sphere((0, 0, 0), 1, b.lambertian(t)), -1, (0, 0, 0))
    p = sc.perlins[0]
    for k in ("perm_x", "perm_y", "perm_z"):
        assert sorted(p[k].tolist()) == list(range(256))
    rv = np.asarray(p["ranvec"])
    assert np.all(np.abs(rv) <= 1.0)
    assert not math.isnan(float(rv.sum()))

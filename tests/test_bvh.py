"""World-BVH rebuild (CPU): the SAH tree the device traverses by default must give the same
closest hits as the reference's makeBVH tree (the oracle traverses both with the reference's own
hit/boxRayIntersect), and must be refused for trees that hold media."""
import numpy as np
import pytest

import pyoracle
import rtamd


def _rays(rng, n, center, spread, target):
    o = np.array(center) + rng.normal(0, spread, (n, 3))
    d = np.array(target) - o + rng.normal(0, 2.0, (n, 3))
    return np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)


@pytest.mark.parametrize("name,center,spread,target,param", [
    ("random_book_one", (13.0, 2.0, 3.0), 3.0, (0.0, 0.0, 0.0), 0),
    ("stress_spheres", (13.0, 2.0, 3.0), 3.0, (0.0, 0.0, 0.0), 3000),
])
def test_rebuilt_tree_gives_identical_closest_hits(name, center, spread, target, param):
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024), param=param)
    rebuilt = rtamd.rebuilt_scene(scene)
    assert rebuilt.desc.world_root != scene.desc.world_root
    rays = _rays(np.random.default_rng(7), 20000, center, spread, target)
    a = pyoracle.closest_hits(scene, rays, 1e-4, np.inf)
    b = pyoracle.closest_hits(rebuilt, rays, 1e-4, np.inf)
    assert a[:, 0].sum() > 1000
    assert np.array_equal(a, b)


def test_rebuilt_tree_is_a_proper_bvh():
    scene, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    rb = rtamd.rebuilt_scene(scene)
    nodes = rb.nodes
    n0 = scene.desc.n_nodes
    root = rb.desc.world_root

    def leaves(i):
        nd = nodes[i]
        if nd["type"] != rtamd.RT_NODE_BVH:
            return [i]
        assert nd["a"] < i and nd["b"] < i
        for ch in (nd["a"], nd["b"]):  # child boxes inside the parent's box
            if nodes[ch]["type"] == rtamd.RT_NODE_BVH:
                assert np.all(nodes[ch]["f"][:3] >= nd["f"][:3]) and np.all(nodes[ch]["f"][3:] <= nd["f"][3:])
        return leaves(nd["a"]) + leaves(nd["b"])

    got = leaves(root)
    assert len(got) == len(set(got))  # every leaf exactly once
    ref = set()

    def ref_leaves(i):
        nd = nodes[i]
        if nd["type"] == rtamd.RT_NODE_BVH and i < n0:
            ref_leaves(nd["a"])
            ref_leaves(nd["b"])
        else:
            ref.add(i)
    ref_leaves(scene.desc.world_root)
    assert set(got) == ref
    # rebuilt nodes carry the ordered flag and a split axis in `c`
    new = nodes[n0:]
    assert np.all((new["c"] & rtamd.RT_BVH_ORDERED) != 0) and np.all((new["c"] & 3) <= 2)


@pytest.mark.parametrize("name", ["cornell_smoke", "next_week_final", "cornell", "three_spheres"])
def test_media_and_small_trees_are_not_rebuilt(name):
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024))
    assert rtamd.rebuilt_scene(scene).desc.world_root == scene.desc.world_root


@pytest.mark.parametrize("name,param", [("random_book_one", 0), ("stress_spheres", 3000), ("cornell", 0),
                                        ("three_spheres", 0)])
def test_wide_tree_covers_leaves_and_contains_boxes(name, param):
    """rt_wide_bvh (the device walk's 4-wide tree): every leaf of the binary world tree exactly
    once, fp32 child boxes containing the leaf's fp64 bounding box (spheres: centre +- r, as
    boundingBox) and every box below them, child ids valid and increasing, stack bound sound."""
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024), param=param)
    rb = rtamd.rebuilt_scene(scene)
    nodes = rb.nodes
    wide, need = rtamd.wide_bvh(rb)
    assert len(wide) >= 1 and need >= 1
    seen = []

    def walk(w, depth_push):
        rec = wide[w]
        kids = []
        for k in range(4):
            lo = rec["lo"][:, k].astype(np.float64)
            hi = rec["hi"][:, k].astype(np.float64)
            c = int(rec["child"][k])
            if np.any(lo > hi):  # unused slot: empty box over a leaf of this node
                assert np.all(np.isinf(lo)) and np.all(np.isinf(hi)) and c < 0
                continue
            kids.append(k)
            if c >= 0:
                assert c > w
                sub = wide[c]
                for kk in range(4):
                    slo, shi = sub["lo"][:, kk].astype(np.float64), sub["hi"][:, kk].astype(np.float64)
                    if np.all(slo <= shi):
                        assert np.all(slo >= lo) and np.all(shi <= hi)
            else:
                leaf = ~c
                seen.append(leaf)
                nd = nodes[leaf]
                if nd["type"] == rtamd.RT_NODE_SPHERE:
                    cen, rad = nd["f"][:3], nd["f"][3]
                    assert np.all(lo <= cen - rad) and np.all(hi >= cen + rad)
        assert kids
        # the nearest accepted child is entered, the others wait on the stack
        deepest = 0
        for k in kids:
            c = int(rec["child"][k])
            if c >= 0:
                deepest = max(deepest, walk(c, 0))
        return len(kids) - 1 + deepest

    assert walk(0, 0) <= need

    def bin_leaves(i):
        nd = nodes[i]
        if nd["type"] == rtamd.RT_NODE_BVH:
            return bin_leaves(nd["a"]) + bin_leaves(nd["b"])
        return [i]
    assert sorted(seen) == sorted(bin_leaves(rb.desc.world_root))
    print(f"{name}: {len(set(seen))} leaves, {len(wide)} wide nodes, stack bound {need}")

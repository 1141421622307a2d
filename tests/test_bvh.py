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


@pytest.mark.parametrize("name", ["cornell_smoke", "cornell", "three_spheres"])
def test_small_trees_are_not_rebuilt(name):
    """Worlds of < 16 leaves keep the caller's tree (media worlds: its unfolded copy, every medium
    occurrence its own keyed record; the topology is the caller's)."""
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024))
    assert not rtamd.prepare_scene(scene)["rebuilt_bvh"]
    rb = rtamd.rebuilt_scene(scene)
    nodes = rb.nodes
    if name != "cornell_smoke":
        assert rb.desc.world_root == scene.desc.world_root
    assert not np.any(nodes["c"][nodes["type"] == rtamd.RT_NODE_BVH] & rtamd.RT_BVH_ORDERED)


def _earth():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "earthmap_rgb8.npz"))["rgb"]


def _medium_occurrences(nodes, i, out):
    """The medium records reached from node i in the walk's preorder (BVH left first, into frames)."""
    nd = nodes[i]
    t = int(nd["type"])
    if t == rtamd.RT_NODE_CONSTANT_MEDIUM:
        out.append(i)
    elif t == rtamd.RT_NODE_BVH:
        _medium_occurrences(nodes, int(nd["a"]), out)
        _medium_occurrences(nodes, int(nd["b"]), out)
    elif t in (rtamd.RT_NODE_TRANSLATE, rtamd.RT_NODE_ROTATE):
        _medium_occurrences(nodes, int(nd["a"]), out)
    return out


@pytest.mark.parametrize("name", ["next_week_final", "cornell_smoke"])
def test_media_are_unfolded_and_keyed(name):
    """rt_rebuild_bvh (the upload's tree): the caller's records untouched (appended only); every medium
    occurrence of the caller's tree — preorder, BVH left first, BVHNode h h and shared sub-trees counted
    once per path — is its own record with f[1] = its preorder rank + 1 (the tier-B draw key); the
    device's tree reaches exactly those keyed records, each once; the same medium records (boundary,
    density, phase material)."""
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024), earth=_earth() if name == "next_week_final" else None)
    rb = rtamd.rebuilt_scene(scene)
    old, new = scene.nodes, rb.nodes
    n0 = scene.desc.n_nodes
    assert np.array_equal(new[:n0], old)
    ref = _medium_occurrences(old, scene.desc.world_root, [])
    dev = _medium_occurrences(new, rb.desc.world_root, [])
    assert len(ref) >= 2 and len(dev) == len(ref)
    keys = sorted(int(new[i]["f"][1]) for i in dev)
    assert keys == list(range(1, len(ref) + 1)) and len(set(dev)) == len(dev)
    by_key = {int(new[i]["f"][1]): i for i in dev}
    for rank, i in enumerate(ref):
        j = by_key[rank + 1]
        assert (new[j]["f"][0] == old[i]["f"][0] and new[j]["a"] == old[i]["a"] and new[j]["b"] == old[i]["b"])


def test_media_world_is_rebuilt_whole():
    """next_week_final (two ConstantMedium, a Translate/Rotate frame over 1000 spheres): with keyed
    media the world keeps no skeleton above them — its two media are hoisted into a chain of
    RT_BVH_MEDIA_FIRST nodes (medium left, the rest right), below which an SAH (RT_BVH_ORDERED) tree
    spans every other leaf, and the frame's inner tree is re-bounded too; the mixed walk then takes one
    4-wide tree below the chain (rt_prepare_scene: mixed_wide)."""
    scene, _ = rtamd.make_scene("next_week_final", rtamd.randGen(1024), earth=_earth())
    rb = rtamd.rebuilt_scene(scene)
    nodes = rb.nodes
    root = rb.desc.world_root
    media = []
    while nodes[root]["type"] == rtamd.RT_NODE_BVH and nodes[root]["c"] & rtamd.RT_BVH_MEDIA_FIRST:
        assert nodes[root]["c"] & rtamd.RT_BVH_ORDERED
        media.append(int(nodes[root]["a"]))
        root = int(nodes[root]["b"])
    assert len(media) == 2 and all(nodes[m]["type"] == rtamd.RT_NODE_CONSTANT_MEDIUM for m in media)
    assert sorted(int(nodes[m]["f"][1]) for m in media) == [1, 2]  # (keyed occurrences)
    assert nodes[root]["type"] == rtamd.RT_NODE_BVH and nodes[root]["c"] & rtamd.RT_BVH_ORDERED
    assert not (nodes[root]["c"] & rtamd.RT_BVH_MEDIA_FIRST)
    frames = [i for i in range(len(nodes)) if nodes[i]["type"] == rtamd.RT_NODE_TRANSLATE and i >= scene.desc.n_nodes]
    assert frames  # the 1000-sphere frame copied with its inner tree re-bounded
    inner = nodes[int(nodes[int(nodes[frames[-1]]["a"])]["a"])]
    assert inner["type"] == rtamd.RT_NODE_BVH and inner["c"] & rtamd.RT_BVH_ORDERED
    info = rtamd.prepare_scene(scene)
    assert info["rebuilt_bvh"] and info["mixed_wide"] and info["n_wide_nodes"] > 300


@pytest.mark.parametrize("name", ["next_week_final", "cornell_smoke"])
def test_skeleton_gives_the_references_closest_hits_and_draws(name):
    """The oracle's hit recursion (tier-B semantics: keyed medium draws, unbounded medium candidates)
    over the device's tree and over the caller's tree: every closest hit identical, medium hits
    included — the keys follow the occurrences (f[1] on the device's records, preorder ranks on the
    caller's), not the order the walk reaches them in."""
    scene, _ = rtamd.make_scene(name, rtamd.randGen(1024), earth=_earth() if name == "next_week_final" else None)
    rb = rtamd.rebuilt_scene(scene)
    rng = np.random.default_rng(11)
    n = 20000
    if name == "next_week_final":
        o = np.array([478.0, 278.0, -600.0]) + rng.normal(0, 30, (n, 3))
        d = np.array([-200.0, 0.0, 600.0]) - np.array([478.0, 278.0, -600.0]) + rng.normal(0, 250, (n, 3))
    else:
        o = rng.uniform(20, 530, (n, 3))
        d = rng.normal(0, 1, (n, 3))
    rays = np.concatenate([o, d, rng.uniform(0, 1, (n, 1))], axis=1)
    a = pyoracle.closest_hits(scene, rays, 1e-4, np.inf, seed=5)
    b = pyoracle.closest_hits(rb, rays, 1e-4, np.inf, seed=5)
    assert a[:, 0].sum() > n // 4
    assert np.array_equal(a, b)


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


def _spine_scene(n=45):
    """Skewed world: n unit spheres in a row at x = -2^k. The SAH rebuild's centroid bins put all
    but the far sphere in bin 0 at every level, so the rebuilt tree is a deep spine."""
    b = rtamd.Builder(rtamd.randGen(1024))
    mat = b.lambertian(b.constantColor(0.3, 0.6, 0.2))
    ids = [b.sphere((-(2.0 ** k), 0.0, 0.0), 0.5, mat) for k in range(n)]
    world = b.makeBVH((0.0, 1.0), ids)
    return b.finish(world, -1, (0.7, 0.8, 0.9))


def _walk_need(nodes, node, signs, memo):
    """Deepest stack the walk (rt_trace.h traverse / walk_step) reaches below `node` for a ray
    whose direction has the given component signs, every box accepted (the worst case)."""
    key = node
    if key in memo:
        return memo[key]
    nd = nodes[node]
    t = int(nd["type"])
    if t == rtamd.RT_NODE_BVH:
        c = int(nd["c"])
        flip = (c & rtamd.RT_BVH_ORDERED) != 0 and not (c & rtamd.RT_BVH_MEDIA_FIRST) and signs[c & 3] < 0
        first, second = (int(nd["b"]), int(nd["a"])) if flip else (int(nd["a"]), int(nd["b"]))
        r = max(1 + _walk_need(nodes, first, signs, memo), _walk_need(nodes, second, signs, memo))
    elif t in (rtamd.RT_NODE_TRANSLATE, rtamd.RT_NODE_ROTATE):
        inner = _walk_need(nodes, int(nd["a"]), signs, memo)
        chain = _is_chain(nodes, int(nd["a"]))
        r = 0 if chain else 1 + inner
    else:
        r = 0
    memo[key] = r
    return r


def _is_chain(nodes, i):
    t = int(nodes[i]["type"])
    if t in (rtamd.RT_NODE_TRANSLATE, rtamd.RT_NODE_ROTATE):
        return _is_chain(nodes, int(nodes[i]["a"]))
    return t in (rtamd.RT_NODE_SPHERE, rtamd.RT_NODE_MOVING_SPHERE, rtamd.RT_NODE_RECT_XY, rtamd.RT_NODE_RECT_XZ,
                 rtamd.RT_NODE_RECT_YZ, rtamd.RT_NODE_CUBOID)


def _left_first_bound(nodes, node, memo):
    """The bound the validator used before ordered nodes were accounted for."""
    if node in memo:
        return memo[node]
    nd = nodes[node]
    r = 0
    if int(nd["type"]) == rtamd.RT_NODE_BVH:
        r = max(1 + _left_first_bound(nodes, int(nd["a"]), memo), _left_first_bound(nodes, int(nd["b"]), memo))
    memo[node] = r
    return r


@pytest.mark.parametrize("name,param", [("random_book_one", 0), ("stress_spheres", 2000), ("stress_spheres", 20000),
                                        ("random", 0), ("cornell", 0), ("next_week_final", 0), ("spine", 0)])
def test_stack_bound_covers_every_ray_direction(name, param):
    """rt_tree_stack_need (the bound rt_upload_scene sizes the LDS stacks with) is at least the
    deepest stack the walk reaches over all 8 direction-sign combinations, on the tree the device
    walks (the SAH rebuild where it applies) and on the caller's tree (the tie redo walk)."""
    import itertools
    if name == "spine":
        scene = _spine_scene()
    else:
        scene, _ = rtamd.make_scene(name, rtamd.randGen(1024), param=param)
    rb = rtamd.rebuilt_scene(scene)
    for sc in (rb, scene):
        nodes = sc.nodes
        bound = rtamd.tree_stack_need(sc)
        worst = max(_walk_need(nodes, sc.desc.world_root, s, {}) for s in itertools.product((1, -1), repeat=3))
        assert worst <= bound, (name, worst, bound)
        assert bound <= 30  # RT_STACK - 2: upload admits it
    if name == "spine":
        # the rebuilt spine is where left-first accounting fell short
        nodes = rb.nodes
        worst = max(_walk_need(nodes, rb.desc.world_root, s, {}) for s in itertools.product((1, -1), repeat=3))
        assert rb.desc.world_root != scene.desc.world_root
        assert _left_first_bound(nodes, rb.desc.world_root, {}) < worst

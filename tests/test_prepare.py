"""The host half of rt_upload_scene without a GPU (rt_prepare_scene, ray-tracing_amd/csrc/rt_prepare.cpp):
the library scenes prepare to the device copies DESIGN.md describes, and malformed descriptors are
rejected with RT_E_INVALID / RT_E_UNSUPPORTED instead of reaching a kernel. The same cases run under
AddressSanitizer + UBSan in tests/test_sanitizers.py (tests/c/host_check.cpp)."""
import ctypes as C
import os

import numpy as np
import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EARTH = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"]
F_MEDIA, F_FRAMES = 8, 512


def _scene(name, **kw):
    return rtamd.make_scene(name, rtamd.randGen(1024), earth=EARTH, **kw)[0]


def _variant(scene, nodes=None, materials=None, textures=None, perlins=None, world=None, lights=None):
    """A copy of scene's descriptor with some arrays replaced (numpy structured copies, kept alive)."""
    d = rt_desc = rtamd.rt_scene_desc()
    C.pointer(d)[0] = scene.desc
    keep = []
    for field, arr, ctype, count in (("nodes", nodes, rtamd.rt_node, "n_nodes"),
                                     ("materials", materials, rtamd.rt_material, "n_materials"),
                                     ("textures", textures, rtamd.rt_texture, "n_textures"),
                                     ("perlins", perlins, rtamd.rt_perlin, "n_perlins")):
        if arr is None:
            continue
        buf = (ctype * len(arr)).from_buffer_copy(np.ascontiguousarray(arr).tobytes()) if len(arr) else None
        keep.append(buf)
        setattr(d, field, C.cast(buf, C.POINTER(ctype)) if buf is not None else None)
        setattr(d, count, len(arr))
    if world is not None:
        d.world_root = world
    if lights is not None:
        d.lights_root = lights
    rt_desc._keep = (keep, scene)
    return rt_desc


def _nodes(scene):
    return scene.nodes.view(np.dtype([("f", "<f8", 6), ("type", "<i4"), ("a", "<i4"), ("b", "<i4"), ("c", "<i4")]))


def _code(desc):
    try:
        rtamd.prepare_scene(desc)
        return 0
    except rtamd.RTError as e:
        return int(str(e).split("(")[1].split(")")[0])


def test_library_scenes_prepare_as_designed():
    c2 = rtamd.prepare_scene(_scene("random_book_one"))
    assert c2["rebuilt_bvh"] and not c2["ref_walk"] and c2["variant"] == 0
    assert c2["n_leaves"] == 486 and 150 < c2["n_wide_nodes"] < 300
    c4 = rtamd.prepare_scene(_scene("next_week_final"))
    assert c4["mixed_wide"] and c4["ref_walk"] and c4["features"] & F_MEDIA and c4["features"] & F_FRAMES
    ref = rtamd.prepare_scene(_scene("next_week_final"), reference_bvh=True)
    assert not ref["rebuilt_bvh"] and not ref["mixed_wide"] and ref["n_wide_nodes"] == 0
    for name in ("three_spheres", "cornell", "cornell_smoke", "two_perlin_spheres", "simple_light", "earth",
                 "two_spheres", "random"):
        info = rtamd.prepare_scene(_scene(name))
        assert info["replace_ok"] and info["n_nodes"] >= _scene(name).desc.n_nodes


def _bvh_ids(nodes):
    return [i for i in range(len(nodes)) if nodes["type"][i] == 0]


def test_ordered_node_with_internal_bits_is_rejected():
    """an RT_BVH_ORDERED node may carry only its split axis in c; RT_WROOT (0x20000000) and
    a stray wide-root index are the upload's own tags."""
    s = _scene("next_week_final")
    for extra in (0x20000000, 0x20000000 | (5 << 2), 3, 1 << 10):
        n = _nodes(s).copy()
        i = _bvh_ids(n)[-1]
        n["c"][i] = 0x40000000 | extra
        assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1, hex(extra)
    for axis in (0, 1, 2):  # the legal forms
        n = _nodes(s).copy()
        n["c"][_bvh_ids(n)[-1]] = 0x40000000 | axis
        assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == 0


def test_ordered_node_in_lights_tree_is_rejected():
    s = _scene("cornell")
    n = _nodes(s).copy()
    lights = s.desc.lights_root
    if n["type"][lights] != 0:
        pytest.skip("cornell lights root is not a BVH node")
    n["c"][lights] = 0x40000000
    assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1


def test_malformed_topology_is_rejected():
    s = _scene("random_book_one")
    n0 = _nodes(s)
    root = s.desc.world_root
    cases = []
    n = n0.copy(); n["a"][root] = root; cases.append(n)            # self loop
    n = n0.copy(); n["b"][root] = root + 5; cases.append(n)        # child after parent
    n = n0.copy(); n["a"][root] = -3; cases.append(n)              # negative child
    n = n0.copy(); n["c"][root] = 0; cases.append(n)               # BVH size 0
    n = n0.copy(); n["type"][root] = 99; cases.append(n)           # unknown type
    n = n0.copy(); n["type"][root] = 0x100; cases.append(n)        # a device-only type flag
    sph = int(np.nonzero(n0["type"] == 1)[0][0])
    n = n0.copy(); n["a"][sph] = 10 ** 6; cases.append(n)          # material out of range
    for n in cases:
        assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1
    assert _code(_variant(s, world=len(n0))) == -1
    assert _code(_variant(s, lights=len(n0))) == -1


def test_payload_record_is_never_a_child():
    s = _scene("random")  # moving spheres: EXT records follow them
    n0 = _nodes(s)
    ext = int(np.nonzero(n0["type"] == 11)[0][0])
    bvh = [i for i in _bvh_ids(n0) if i > ext][0]
    n = n0.copy()
    n["a"][bvh] = ext
    assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1
    assert _code(_variant(s, world=ext)) == -1
    n = n0.copy()  # a moving sphere that lost its payload record
    ms = ext - 1
    n["type"][ext] = 10
    assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1 or n0["type"][ms] != 2


def test_bad_textures_materials_and_perlin_tables():
    s = _scene("two_perlin_spheres")
    p = s.perlins.copy()
    raw = np.frombuffer(p.tobytes(), dtype=np.uint8).copy()
    perm_off = 256 * 3 * 8
    perm = raw[perm_off:perm_off + 4].view("<i4")
    perm[0] = 256
    assert _code(_variant(s, perlins=raw.view(p.dtype))) == -1
    t = s.textures.copy().view(np.dtype([("type", "<i4"), ("a", "<i4"), ("b", "<i4"), ("c", "<i4"), ("f", "<f8", 4)]))
    bad = t.copy(); bad["type"][0] = 7
    assert _code(_variant(s, textures=bad.view(s.textures.dtype))) == -1
    pi = int(np.nonzero(t["type"] == 2)[0][0])
    bad = t.copy(); bad["a"][pi] = 5
    assert _code(_variant(s, textures=bad.view(s.textures.dtype))) == -1
    m = s.materials.copy().view(np.dtype([("type", "<i4"), ("tex", "<i4"), ("param", "<f8")]))
    bad = m.copy(); bad["tex"][0] = 1000
    assert _code(_variant(s, materials=bad.view(s.materials.dtype))) == -1
    bad = m.copy(); bad["type"][0] = 9
    assert _code(_variant(s, materials=bad.view(s.materials.dtype))) == -1


def test_checker_children_must_precede_and_images_stay_in_pool():
    s = _scene("random")  # the checker ground texture
    t = s.textures.copy().view(np.dtype([("type", "<i4"), ("a", "<i4"), ("b", "<i4"), ("c", "<i4"), ("f", "<f8", 4)]))
    ci = int(np.nonzero(t["type"] == 1)[0][0])
    bad = t.copy(); bad["a"][ci] = ci
    assert _code(_variant(s, textures=bad.view(s.textures.dtype))) == -1
    e = _scene("earth")
    t = e.textures.copy().view(bad.dtype)
    ii = int(np.nonzero(t["type"] == 3)[0][0])
    for field, val in (("b", int(t["b"][ii]) + 1), ("a", 3)):
        bad = t.copy(); bad[field][ii] = val
        assert _code(_variant(e, textures=bad.view(e.textures.dtype))) == -1


def test_medium_keys_all_or_none_and_distinct():
    """tier-B medium draws are keyed per occurrence (include/rt.h; f[1] = key + 1 when the caller
    sets it, else the occurrence's preorder rank). Caller keys are accepted only on every occurrence of the
    world and only when distinct: a keyed record reached twice, or a caller key equal to an unkeyed
    occurrence's rank, would make two occurrences draw the same numbers."""
    s = _scene("next_week_final")
    n0 = _nodes(s)
    med = [int(i) for i in np.nonzero(n0["type"] == 9)[0]]
    assert len(med) == 2
    assert _code(s.desc) == 0

    def with_keys(vals):
        n = n0.copy()
        for i, v in zip(med, vals):
            n["f"][i, 1] = v
        return _variant(s, nodes=n.view(s.nodes.dtype))

    assert _code(with_keys([1.0, 2.0])) == 0      # every occurrence keyed, distinct
    assert _code(with_keys([7.0, 3.0])) == 0
    assert _code(with_keys([1.0, 0.0])) == -1     # keyed and unkeyed mixed (key 0 = the other's rank)
    assert _code(with_keys([0.0, 5.0])) == -1
    assert _code(with_keys([2.0, 2.0])) == -1     # one key twice
    assert _code(with_keys([1.5, 2.0])) == -1     # not an integer
    assert _code(with_keys([2.0 ** 32, 1.0])) == -1  # beyond the counter word's 31 bits
    # BVHNode h h over a keyed medium (src/Lib.hs:948): one record reached along two paths
    n = n0.copy()
    n["f"][med[0], 1] = 1.0
    n["f"][med[1], 1] = 2.0
    parent = [i for i in _bvh_ids(n) if n["a"][i] == med[0] or n["b"][i] == med[0]][0]
    n["a"][parent] = n["b"][parent] = med[0]
    assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) == -1
    # the unfolded array (rt_rebuild_bvh: every occurrence keyed by its rank) prepares again as is
    rb = rtamd.rebuilt_scene(s)
    assert _code(rb.desc) == 0
    assert (_nodes(rb)["f"][_nodes(rb)["type"] == 9][:, 1] >= 1).sum() >= 2


def test_random_mutations_never_crash():
    """Seeded field mutations of valid descriptors: every call returns RT_OK or an error code (the
    sanitizer build runs the same loop natively, tests/c/host_check.cpp)."""
    rng = np.random.default_rng(5)
    for name in ("random_book_one", "next_week_final", "cornell_smoke"):
        s = _scene(name)
        n0 = _nodes(s)
        for _ in range(150):
            n = n0.copy()
            for _ in range(int(rng.integers(1, 4))):
                i = int(rng.integers(0, len(n)))
                fld = ("type", "a", "b", "c")[int(rng.integers(0, 4))]
                n[fld][i] = int(rng.choice([-1, 0, 1, 2, 3, 11, i, i + 1, len(n), 0x40000000 | 2, 0x2fffffff]))
            assert _code(_variant(s, nodes=n.view(s.nodes.dtype))) in (0, -1, -4)

"""C-ABI checks without a GPU: the library loads, exports exactly what include/rt.h declares,
validates arguments, and writes the reference's P3 format."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "rt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    inline = set(re.findall(r"static\s+inline\s+\w+\s+(rt_[a-z0-9_]+)\s*\(", src))  # header-only helpers
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)) - inline)


def test_every_declared_symbol_is_exported():
    L = rtamd.lib()
    declared = _declared()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(rtamd.EXPORTED) == declared


def test_abi_version():
    assert rtamd.lib().rt_abi_version() == 1


def test_struct_sizes_match_header():
    assert C.sizeof(rtamd.rt_node) == 64
    assert C.sizeof(rtamd.rt_scene_desc) == 112
    assert C.sizeof(rtamd.rt_render_params) == 48
    assert C.sizeof(rtamd.rt_launch_info) == 56
    assert rtamd.rt_launch_info.wide_nodes.offset == 44  # (round 3: was _pad)
    assert rtamd.rt_launch_info.chunk_batches.offset == 48  # (round 4)
    assert C.sizeof(rtamd.rt_frame_timing) == 8 + 8 * rtamd.RT_MAX_DEVICES + 24  # (round 5)


def test_param_validation_without_gpu():
    with pytest.raises(rtamd.RTError):
        rtamd.shard_geometry(rtamd.make_params(0, 10, 1, 1))
    for tile in (12, -8, 264, 65536):  # (tile*tile must stay a 32-bit work-item count)
        with pytest.raises(rtamd.RTError):
            rtamd.shard_geometry(rtamd.make_params(10, 10, 1, 1, tile=tile))
    assert rtamd.shard_geometry(rtamd.make_params(10, 10, 1, 1, tile=256))[0] == 1
    with pytest.raises(rtamd.RTError):
        rtamd.shard_geometry(rtamd.make_params(10, 10, 1, 1, shard_rank=2, shard_count=2))
    for count in (0, 1):  # an unsharded launch has only rank 0 (a stray rank shifted the tile map)
        with pytest.raises(rtamd.RTError):
            rtamd.shard_geometry(rtamd.make_params(10, 10, 1, 1, shard_rank=1, shard_count=count))
    tt, per, slab = rtamd.shard_geometry(rtamd.make_params(1200, 800, 1, 1, tile=16, shard_count=8))
    assert tt == 75 * 50 and per == (3750 + 7) // 8 and slab == per * 256


def test_ppm_matches_printrow():
    """P3 / "W H" / 255, then one line per row of space-separated components (src/Lib.hs:299-305)."""
    rgb = np.random.default_rng(0).integers(0, 256, (3, 4, 3), dtype=np.uint8)
    txt = rtamd.write_ppm(rgb).decode()
    lines = txt.split("\n")
    assert lines[0] == "P3" and lines[1] == "4 3" and lines[2] == "255"
    for r in range(3):
        assert lines[3 + r] == " ".join(str(int(v)) for v in rgb[r].reshape(-1))
    assert txt.endswith("\n") and len(lines) == 3 + 3 + 1


def test_tile_map_is_a_partition():
    """Across shards, every pixel is owned exactly once (the gather is a permutation)."""
    for W, H, tile, n in [(1200, 800, 16, 8), (97, 61, 16, 3), (200, 100, 8, 2), (33, 17, 32, 5)]:
        seen = np.zeros(W * H, dtype=np.int64)
        for r in range(n):
            m = rtamd.shard_pixel_map(rtamd.make_params(W, H, 1, 1, tile=tile, shard_rank=r, shard_count=n))
            np.add.at(seen, m[m >= 0], 1)
        assert (seen == 1).all()


def test_render_without_device_fails_loudly():
    """No CPU fallback: creating a device context on a box with no GPU raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rtamd.RTError):
        rtamd.Context(0)


def test_multi_device_ctx_validation_without_gpu():
    """rt_create_multi checks its device list before touching a device: 1..RT_MAX_DEVICES devices; with
    no GPU it fails loudly like rt_create (no CPU fallback). The library links RCCL for the gather."""
    L = rtamd.lib()
    h = C.c_void_p()
    for n in (0, -1, rtamd.RT_MAX_DEVICES + 1):
        assert L.rt_create_multi(n, None, C.byref(h)) == rtamd.RT_E_INVALID and not h.value
    import torch
    if not torch.cuda.is_available():
        assert L.rt_create_multi(1, None, C.byref(h)) < 0 and not h.value
        with pytest.raises(rtamd.RTError):
            rtamd.Context(devices=[0])
    assert L.rt_ctx_devices(None, None, None, 0) == rtamd.RT_E_INVALID
    import subprocess
    ldd = subprocess.run(["ldd", rtamd.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl.so.1" in ldd


def test_pfm_float_dump_round_trip():
    """rt_write_pfm: PFM float32 bottom row first, and the lossless PF64 variant;
    NaN pixels stay NaN."""
    lin = np.random.default_rng(1).random((5, 7, 3))
    lin[2, 3] = np.nan
    pf = rtamd.write_pfm(lin)
    assert pf.startswith(b"PF\n7 5\n-1.0\n") and len(pf) == len(b"PF\n7 5\n-1.0\n") + 5 * 7 * 3 * 4
    first = np.frombuffer(pf[len(b"PF\n7 5\n-1.0\n"):][:7 * 3 * 4], dtype="<f4")
    assert np.array_equal(first, lin[4].reshape(-1).astype(np.float32))  # bottom row first
    back = rtamd.read_pfm(pf)
    assert np.array_equal(back, lin.astype(np.float32).astype(np.float64), equal_nan=True)
    assert np.array_equal(rtamd.read_pfm(rtamd.write_pfm(lin, f64=True)), lin, equal_nan=True)

"""CPU pins of the bench-band fixtures (tests/golden/bench_bands.npz) and of bench.py's host-side
accounting: the oracle reproduces a row of each cheap band bit for bit (so the fixtures stay the
oracle's output), and bench.sample_chunk mirrors rt_sample_chunk (include/rt.h)."""
import os

import numpy as np
import pytest

import bench
import pyoracle
import rtamd

HERE = os.path.dirname(os.path.abspath(__file__))
B = np.load(os.path.join(HERE, "golden", "bench_bands.npz"))


@pytest.mark.parametrize("key,scene,cam,earth", [("c2", "random_book_one", "random_scene", False),
                                                 ("c3", "cornell", "cornell", False),
                                                 ("c4s", "next_week_final", "next_week", True),
                                                 ("c2z", "random_book_one", "random_scene", False)])
def test_oracle_reproduces_band_row(key, scene, cam, earth):
    W, H, spp, depth, seed, r0, flags = [int(x) for x in B[f"{key}_frame"]]
    e = np.load(os.path.join(HERE, "golden", "earthmap_rgb8.npz"))["rgb"] if earth else None
    sc, _ = rtamd.make_scene(scene, rtamd.randGen(1024), earth=e)
    p = rtamd.make_params(W, H, spp, depth, rtamd.RT_RNG_PHILOX, seed=seed, flags=flags)
    rgb, lin, _, _ = pyoracle.render(sc, rtamd.camera(cam, W, H), p, rows=(r0, r0 + 1))
    assert np.array_equal(rgb[0], B[f"{key}_rgb"][0])
    assert np.array_equal(lin[0], B[f"{key}_lin"][0], equal_nan=True)


def test_nan_zero_keeps_the_finite_part():
    """RT_FLAG_NAN_ZERO on the oracle: pixels without a NaN sample are unchanged, the others finite."""
    sc, _ = rtamd.make_scene("three_spheres", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 40, 20)
    a = pyoracle.render(sc, cam, rtamd.make_params(40, 20, 4, 10, rtamd.RT_RNG_PHILOX, seed=5))[1]
    b = pyoracle.render(sc, cam, rtamd.make_params(40, 20, 4, 10, rtamd.RT_RNG_PHILOX, seed=5,
                                                   flags=rtamd.RT_FLAG_NAN_ZERO))[1]
    fin = ~np.isnan(a)
    assert np.isnan(a).any() and fin.any() and not np.isnan(b).any()
    assert np.array_equal(a[fin], b[fin])


def test_sample_chunk_mirror():
    for (px, spp), ch in {(768, 33): 1, (4096, 600): 3, (12288, 700): 8, (7680, 1200): 9, (65536, 130): 8, (19200, 1100): 9,
                          (19200, 2200): 18, (960000, 500): 8, (360000, 1000): 8, (640000, 1000): 8,
                          (8294400, 2000): 16, (20000, 10): 1, (8294400, 4): 4}.items():
        assert bench.sample_chunk(px, spp) == ch


def test_algorithmic_offchip_bytes_c2():
    cfg = bench.CONFIGS["c2"]
    sc, _ = rtamd.make_scene(cfg["scene"], rtamd.randGen(1024))
    p = rtamd.make_params(cfg["W"], cfg["H"], cfg["spp"], cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024)
    off = bench.algorithmic_offchip_bytes(cfg, p, sc)
    slab = 75 * 50 * 256  # 16x16 tiles of the 1200x800 frame
    assert off["chunk_sums"] == slab * 63 * 24 and off["image"] == slab * 3
    assert off["total"] == off["chunk_sums"] + off["image"] + off["scene"] and off["scene"] > 64 * 997


def test_cpu_baseline_threads_follow_affinity(monkeypatch):
    class A:
        cpu_threads = 0
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n, c = bench.cpu_threads(A())
    assert n == min(3, len(os.sched_getaffinity(0))) and c["nproc"] == os.cpu_count()
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads(A())[0] == len(os.sched_getaffinity(0))

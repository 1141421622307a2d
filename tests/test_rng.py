"""RNG known-answer tests (CPU).

Pinned: Philox4x32-10 against the Random123 published vectors; splitmix's variant-13 mixer against
Vigna's splitmix64 reference sequence. UNPINNED: the full random-1.2.0/splitmix-0.1 stream as GHC
produces it (no GHC here) — instead three independent restatements (oracle C,
product C++, pure Python) must agree bit for bit.
"""
import math

import numpy as np
import pytest

import pyoracle
import rtamd
import scenes_ref

# Random123 kat_vectors: philox4x32 10 rounds
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,expect", PHILOX_KAT)
def test_philox_kat(ctr, key, expect):
    assert pyoracle.philox(ctr, key) == expect


def test_splitmix_variant13_mixer_pinned():
    # Vigna's splitmix64.c (output = Stafford mix13), seed 1234567
    s, out = 1234567, []
    for _ in range(5):
        s = (s + 0x9E3779B97F4A7C15) & scenes_ref.M64
        out.append(scenes_ref.mix64v13(s))
    assert out == [6457827717110365317, 3203168211198807973, 9817491932198370423, 4593380528125082431,
                   16408922859458223821]


@pytest.mark.parametrize("seed", [0, 1, 1024, 1025, 2 ** 31 - 1, -5, 123456789])
def test_mkstdgen_three_restatements_agree(seed):
    a = pyoracle.mk_smgen(seed)
    b = rtamd.randGen(seed)
    c = tuple(scenes_ref.mk_smgen(seed))
    assert a == b == c
    assert a[1] & 1 == 1  # gamma is odd


def test_draw_streams_agree():
    g = rtamd.randGen(1024)
    ours = []
    gg = g
    for _ in range(64):
        x, gg = rtamd.randomDouble(gg)
        ours.append(x)
    ref, _ = pyoracle.draws(g, 64)
    py = scenes_ref.Gen(g)
    assert ours == ref == [py.D() for _ in range(64)]
    assert all(0.0 <= x <= 1.0 for x in ours)


def test_word_to_draw_edges():
    L = pyoracle.lib()
    assert L.oracle_word_to_draw(0) == 1.0  # 1 - 0/2^64
    assert L.oracle_word_to_draw(2 ** 64 - 1) == 0.0  # (double)(2^64-1) rounds to 2^64
    assert L.oracle_word_to_draw(2 ** 63) == 0.5


def test_scale_color_semantics():
    """scaleColor = floor (256 * clamp (0, 0.999) (sqrt x)); NaN -> 0 (src/Lib.hs:287-288)."""
    L = pyoracle.lib()
    assert L.oracle_scale_color(float("nan")) == 0
    assert L.oracle_scale_color(float("inf")) == 255
    assert L.oracle_scale_color(-1.0) == 0
    assert L.oracle_scale_color(1.0) == 255
    assert L.oracle_scale_color(0.25) == 128
    assert L.oracle_scale_color(0.0) == 0


@pytest.mark.parametrize("y,x", [(1.0, 1.0), (1.0, -1.0), (-1.0, -1.0), (-1.0, 1.0), (0.0, -1.0), (-0.0, -1.0),
                                 (0.0, 0.0), (-0.0, -0.0), (0.0, -0.0), (1.0, 0.0), (-1.0, 0.0), (0.3, -2.5)])
def test_ghc_atan2_matches_ieee_quadrants(y, x):
    """GHC's RealFloat atan2 (atan-based) agrees with libm atan2 in sign/quadrant and to ~1 ulp."""
    got = pyoracle.lib().oracle_ghc_atan2(y, x)
    want = math.atan2(y, x)
    assert math.copysign(1.0, got) == math.copysign(1.0, want)
    assert abs(got - want) <= 4e-16 * max(1.0, abs(want))


def test_tier_b_stream_layout():
    """Tier B: draw 2k and 2k+1 of (pixel, sample) come from Philox block k, words (0,1) and (2,3)."""
    key = 1024
    o = pyoracle.philox([3, 7, 11, 0], [key & 0xFFFFFFFF, key >> 32])
    w0 = o[0] | (o[1] << 32)
    w1 = o[2] | (o[3] << 32)
    d0 = 1.0 - float(w0) / 2.0 ** 64
    d1 = 1.0 - float(w1) / 2.0 ** 64
    assert 0.0 <= d0 <= 1.0 and 0.0 <= d1 <= 1.0 and d0 != d1
    assert np.isfinite([d0, d1]).all()

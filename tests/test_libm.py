"""include/rt_libm.h on the host (the oracle's build of it): the portable transcendentals that
RT_FLAG_SHARED_LIBM makes the device and the oracle share. Accuracy against mpmath (300-bit), IEEE
special values, and closeness to glibc (the reference's libm). The device's bit-identity with this
build is tests/test_gpu_math.py::test_shared_libm_bit_identical_to_host."""
import math

import numpy as np
import pytest

import pyoracle

OPS = {"sin": (12, math.sin), "cos": (13, math.cos), "atan": (14, math.atan), "asin": (15, math.asin),
       "log": (16, math.log)}


@pytest.mark.parametrize("name,lo,hi,max_ulp", [("sin", 0, 2 * math.pi, 1.0), ("cos", 0, 2 * math.pi, 1.0),
                                                ("sin", -3000, 3000, 1.0), ("cos", -3000, 3000, 1.0),
                                                ("atan", -40, 40, 1.5), ("asin", -1, 1, 2.0), ("log", 0, 1, 1.0)])
def test_accuracy_against_mpmath(name, lo, hi, max_ulp):
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 300
    op, glibc = OPS[name]
    rng = np.random.default_rng(11)
    x = rng.uniform(lo, hi, 3000)
    if name == "log":
        x = 1.0 - x  # (0, 1]: the media's draws
    got = pyoracle.shared_libm(op, x)
    f = getattr(mpmath, name)
    worst, glibc_eq = 0.0, 0
    for a, g in zip(x, got):
        ref = f(mpmath.mpf(float(a)))
        worst = max(worst, float(abs(mpmath.mpf(float(g)) - ref) / math.ulp(float(ref))))
        glibc_eq += g == glibc(float(a))
    print(f"{name}[{lo},{hi}]: max {worst:.3f} ulp, equal to glibc {glibc_eq / len(x):.4f}")
    assert worst <= max_ulp and glibc_eq / len(x) >= 0.6


def test_special_values():
    inf, nan = math.inf, math.nan
    x = np.array([0.0, -0.0, inf, -inf, nan, 1.0, -1.0, 5e-324, 2.0])
    s, c = pyoracle.shared_libm(12, x), pyoracle.shared_libm(13, x)
    at, asn, lg = pyoracle.shared_libm(14, x), pyoracle.shared_libm(15, x), pyoracle.shared_libm(16, x)
    sb = np.signbit
    assert s[0] == 0 and not sb(s[0]) and s[1] == 0 and sb(s[1]) and np.isnan(s[2:5]).all() and s[7] == 5e-324
    assert c[0] == 1 and c[1] == 1 and np.isnan(c[2:5]).all()
    assert sb(at[1]) and at[2] == math.pi / 2 and at[3] == -math.pi / 2 and np.isnan(at[4]) and at[5] == math.pi / 4
    assert sb(asn[1]) and asn[5] == math.pi / 2 and asn[6] == -math.pi / 2 and np.isnan(asn[8]) and np.isnan(asn[2])
    assert lg[0] == -inf and lg[1] == -inf and lg[2] == inf and np.isnan(lg[3]) and lg[5] == 0 and np.isnan(lg[6])
    assert abs(lg[7] - math.log(5e-324)) <= 1e-12 and abs(lg[8] - math.log(2.0)) == 0

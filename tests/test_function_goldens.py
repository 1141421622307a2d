"""Per-function golden vectors (tests/golden/function_goldens.npz, make_function_goldens.py): scatter
(every material kind, src/Lib.hs:822-885), htblRandom / htblPdfValue (src/Lib.hs:673-724),
textureValue (src/Lib.hs:496-513) and getRay (src/Lib.hs:1253-1267), one Philox stream per record.

CPU: the oracle reproduces them bit for bit. GPU: the device functions (rt_debug_probe, the same
inlined code the render kernels run) reproduce them — Philox words consumed and the scattered /
specular flags exactly; the doubles bit for bit except through fp64 transcendentals (OCML on the
device, glibc in the oracle, <= 1 ulp apart: sin/cos in the cosine and unit-vector samples, the
sphere-light sample and the Perlin marble; atan/asin are not on these paths), where they must agree
within 1e-12 relative. Discrete flips (a branch on a value that differs by an ulp: the checker's
sign, a Schlick or rejection comparison) may change at most 1 record in 500; each test prints its
exact-match and flip fractions.
"""
import os

import numpy as np
import pytest

import pyoracle
import rtamd

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "function_goldens.npz"))
SEED = 77
CASES = sorted({k[: -len("_in")] for k in G.files if k.endswith("_in")})
FNS = ("htbl_random", "htbl_pdf", "scatter", "texture", "get_ray")


def _split(case):
    for fn in FNS:
        if case.endswith("_" + fn):
            return case[: -len(fn) - 1], fn
    raise ValueError(case)


def _scene(name):
    from make_function_goldens import make_scene
    return make_scene(name)


@pytest.fixture(scope="module", autouse=True)
def _golden_path():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_function_goldens(case):
    name, fn = _split(case)
    sc, cam, _ = _scene(name)
    out = pyoracle.probe(sc, fn, G[case + "_in"], seed=SEED, cam=cam)
    assert np.array_equal(out, G[case + "_out"], equal_nan=True)


# integer-valued columns (exact) per function: flags and Philox words consumed
EXACT = {"scatter": [0, 12, 13], "htbl_random": [3], "htbl_pdf": [1], "texture": [], "get_ray": [7]}


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_device_functions_match_goldens(gpu_ctx, case):
    name, fn = _split(case)
    sc, cam, _ = _scene(name)
    gpu_ctx.upload(sc)
    got = gpu_ctx.probe(fn, G[case + "_in"], seed=SEED, cam=cam)
    ref = G[case + "_out"]
    same_int = np.all(got[:, EXACT[fn]] == ref[:, EXACT[fn]], axis=1) if EXACT[fn] else np.ones(len(ref), bool)
    exact = np.all((got == ref) | (np.isnan(got) & np.isnan(ref)), axis=1)
    with np.errstate(invalid="ignore"):
        close = np.all(np.isclose(got, ref, rtol=1e-12, atol=1e-300, equal_nan=True), axis=1)
    flips = ~(same_int & close)
    print(f"{case}: {len(ref)} records, bit-exact {exact.mean():.4f}, within 1e-12 {close.mean():.4f}, "
          f"flips {int(flips.sum())}")
    assert flips.mean() <= 0.002, f"{int(flips.sum())} of {len(ref)} records differ beyond 1e-12 / in words"
    if fn in ("htbl_pdf", "get_ray"):  # no transcendental on these paths (sqrt and IEEE divisions only)
        assert exact.all(), f"{int((~exact).sum())} records not bit-exact"

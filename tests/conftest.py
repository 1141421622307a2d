"""Shared test setup: import paths, the `gpu` marker, and parity helpers."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ray-tracing_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librtamd.so's HIP path)")


@pytest.fixture(scope="session")
def gpu_ctx():
    import rtamd
    ctx = rtamd.Context(0)
    yield ctx
    ctx.close()


def display(lin):
    """The pre-quantisation value albedoToColor rounds: sqrt(clamp(0, 0.999)) (src/Lib.hs:287-288)."""
    with np.errstate(invalid="ignore"):
        s = np.sqrt(lin)
        return np.where(s < 0, 0.0, np.where(s > 0.999, 0.999, s))


def parity(lin_a, lin_b, rgb_a, rgb_b, tol=1e-3):
    """SURVEY.md 8d metric: per channel |d| <= tol on the displayed float (NaN == NaN), and the
    8-bit bytes. Returns (fraction of channels within tol, fraction of equal bytes, max |d|)."""
    da, db = display(lin_a), display(lin_b)
    both_nan = np.isnan(da) & np.isnan(db)
    with np.errstate(invalid="ignore"):
        d = np.abs(da - db)
    ok = both_nan | (d <= tol)
    dmax = float(np.nanmax(np.where(both_nan, 0.0, d))) if d.size else 0.0
    return float(ok.mean()), float((rgb_a == rgb_b).mean()), dmax

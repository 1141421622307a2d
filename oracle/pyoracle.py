"""ORACLE binding — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke, bench.py cpu_baseline).

ctypes wrapper of oracle/build/liboracle.so, the C restatement of the reference render path
(see oracle/oracle.c header for what it restates and its pinning status). It renders from the same
flattened scene descriptor (include/rt.h) the product consumes.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

COUNTERS = ["world_queries", "box_tests", "sphere_tests", "rect_tests", "other_prims", "scatters", "draws",
            "samples", "light_queries"]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, D, U64 = C.POINTER, C.c_double, C.c_uint64
        L.oracle_render_rows.restype = C.c_int
        L.oracle_render_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(U64), C.c_int, C.c_int,
                                         P(C.c_uint8), P(D), P(U64), C.c_int, P(C.c_int64)]
        L.oracle_closest_hits.restype = C.c_int
        L.oracle_closest_hits.argtypes = [C.c_void_p, P(D), C.c_int, D, D, U64, P(D)]
        L.oracle_mk_smgen.argtypes = [U64, P(U64)]
        L.oracle_next_word64.restype = U64
        L.oracle_next_word64.argtypes = [P(U64)]
        L.oracle_random_double.restype = D
        L.oracle_random_double.argtypes = [P(U64)]
        L.oracle_philox.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.oracle_word_to_draw.restype = D
        L.oracle_word_to_draw.argtypes = [U64]
        L.oracle_scale_color.restype = C.c_uint8
        L.oracle_scale_color.argtypes = [D]
        L.oracle_ghc_atan2.restype = D
        L.oracle_ghc_atan2.argtypes = [D, D]
        L.oracle_num_counters.restype = C.c_int
        L.oracle_probe.restype = C.c_int
        L.oracle_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int, P(D), C.c_int, U64, P(D)]
        L.oracle_exact_trace.restype = C.c_int
        L.oracle_exact_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(U64), C.c_int, P(D), C.c_int,
                                         P(C.c_int)]
        L.oracle_shared_libm.restype = None
        L.oracle_shared_libm.argtypes = [C.c_int, P(D), P(D), C.c_int, P(D)]
        _lib = L
    return _lib


def render(scene, cam, params, col_gens=None, rows=None, nthreads=0, linear=True, counters=False):
    """Render rows [r0, r1) (default: all) of the image. Returns (rgb, linear, gens_out, counters)."""
    W, H = params.width, params.height
    r0, r1 = rows if rows is not None else (0, H)
    n = (r1 - r0) * W
    rgb = np.zeros((r1 - r0, W, 3), dtype=np.uint8)
    lin = np.zeros((r1 - r0, W, 3), dtype=np.float64) if linear else None
    P = C.POINTER
    gi = None
    go = None
    if col_gens is not None:
        gi = np.ascontiguousarray(col_gens, dtype=np.uint64).reshape(-1)
        go = np.zeros((W, 2), dtype=np.uint64)
    cnt = np.zeros(lib().oracle_num_counters(), dtype=np.int64) if counters else None
    rc = lib().oracle_render_rows(
        C.addressof(scene.desc), C.addressof(cam), C.addressof(params),
        gi.ctypes.data_as(P(C.c_uint64)) if gi is not None else None, r0, r1,
        rgb.ctypes.data_as(P(C.c_uint8)), lin.ctypes.data_as(P(C.c_double)) if lin is not None else None,
        go.ctypes.data_as(P(C.c_uint64)) if go is not None else None, int(nthreads),
        cnt.ctypes.data_as(P(C.c_int64)) if cnt is not None else None)
    if rc != 0:
        raise RuntimeError(f"oracle_render_rows failed ({rc})")
    del n
    c = dict(zip(COUNTERS, cnt.tolist())) if cnt is not None else None
    return rgb, lin, go, c


def closest_hits(scene, rays, tmin, tmax, seed=0):
    rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 7)
    out = np.zeros((rays.shape[0], 12), dtype=np.float64)
    P = C.POINTER
    lib().oracle_closest_hits(C.addressof(scene.desc), rays.ctypes.data_as(P(C.c_double)), rays.shape[0], tmin,
                              tmax, seed, out.ctypes.data_as(P(C.c_double)))
    return out


def probe(scene, op, inputs, seed=0, cam=None):
    """oracle_probe: one hot-path function per record (layouts: oracle/oracle.c, include/rt.h)."""
    import rtamd
    k = rtamd.PROBES[op]
    x = np.ascontiguousarray(inputs, dtype=np.float64).reshape(-1, rtamd.PROBE_IN[k])
    out = np.zeros((x.shape[0], rtamd.PROBE_OUT[k]), dtype=np.float64)
    P = C.POINTER
    rc = lib().oracle_probe(C.addressof(scene.desc), C.addressof(cam) if cam is not None else None, k,
                            x.ctypes.data_as(P(C.c_double)), x.shape[0], seed, out.ctypes.data_as(P(C.c_double)))
    if rc != 0:
        raise RuntimeError(f"oracle_probe failed ({rc})")
    return out


def mk_smgen(s):
    g = (C.c_uint64 * 2)()
    lib().oracle_mk_smgen(s & 0xFFFFFFFFFFFFFFFF, g)
    return int(g[0]), int(g[1])


def draws(gen, n):
    g = (C.c_uint64 * 2)(*gen)
    return [lib().oracle_random_double(g) for _ in range(n)], (int(g[0]), int(g[1]))


def words(gen, n):
    g = (C.c_uint64 * 2)(*gen)
    return [int(lib().oracle_next_word64(g)) for _ in range(n)], (int(g[0]), int(g[1]))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox(c, k, o)
    return [int(x) for x in o]


def shared_libm(op, x, y=None):
    """include/rt_libm.h evaluated on the host (op ids as rt_debug_math: 12 sin ... 17 GHC atan2)."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    y = np.zeros_like(x) if y is None else np.ascontiguousarray(y, dtype=np.float64).reshape(-1)
    out = np.zeros_like(x)
    P = C.POINTER
    lib().oracle_shared_libm(op, x.ctypes.data_as(P(C.c_double)), y.ctypes.data_as(P(C.c_double)), x.size,
                             out.ctypes.data_as(P(C.c_double)))
    return out


def exact_trace(scene, cam, params, col_gens, col, cap=1 << 20):
    """oracle_exact_trace: tier A, column `col`, every path segment (10 doubles: row, sample, seg, o, d,
    seed bits) — to compare with the device's rt_debug_exact_trace."""
    gi = np.ascontiguousarray(col_gens, dtype=np.uint64).reshape(-1)
    out = np.zeros((cap, 10), dtype=np.float64)
    n = C.c_int(0)
    P = C.POINTER
    rc = lib().oracle_exact_trace(C.addressof(scene.desc), C.addressof(cam), C.addressof(params),
                                  gi.ctypes.data_as(P(C.c_uint64)), col, out.ctypes.data_as(P(C.c_double)), cap,
                                  C.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle_exact_trace failed ({rc})")
    return out[: n.value].copy()

"""Tier A's agreement with a glibc-hosted reference when each side uses its own libm.

A tier-A column is one serial chain of draws (src/Lib.hs:1491-1523): a last-bit difference in sin, cos,
log, atan, asin or x ** 5 that later flips a branch (a rejection loop, a Dielectric coin, a medium's
distance against the inside length) changes how many numbers the column consumes, and every pixel below
then renders from other draws. The reference's numbers come from its host's libm (GHC calls glibc's on
Linux); the drop-in runRenderAMD (flags 0) evaluates OCML on the device.

This renders one tier-A frame three or four ways — the oracle with glibc, the oracle with include/rt_libm.h
(RT_FLAG_SHARED_LIBM: a second libm on the CPU, the proxy), and with --gpu the device with OCML (the drop-in)
and with rt_libm.h (which must equal the oracle's rt_libm.h render bit for bit) — and reports, against the
glibc render:
  * columns whose end-of-stream generators are equal (the same number of draws consumed),
  * the north-star metric: channels within 1e-3 on the displayed value, bytes equal,
  * per column, the first row whose pixel differs beyond 1e-3: the column's stream diverged in or above
    that row (bit differences alone are the last-bit residue on agreeing streams). With a
    constant rate lam of divergence per sample, a column survives n samples with probability exp(-lam n);
    lam's maximum-likelihood estimate over the columns (censored at the frame's end) predicts the agreement
    at other frame sizes: a pixel at row r is bit-identical while its column has survived (r + 1) * spp
    samples.
One JSON line per comparison (stdout and --out)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ray-tracing_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
import rtamd  # noqa: E402
from conftest import parity  # noqa: E402


def first_diff_rows(lin_a, lin_b):
    """Per column: the first row whose pixel differs beyond the north-star tolerance in any channel (|d| > 1e-3
    on the displayed value, or NaN on one side only), or H when none does. (Bit differences alone are the
    libms' last-bit residue, ~1e-15, on streams that still agree: a column whose stream diverged renders
    other samples from there on, which differ by the Monte-Carlo noise.)"""
    from conftest import display
    da, db = display(lin_a), display(lin_b)
    with np.errstate(invalid="ignore"):
        same = (np.isnan(da) & np.isnan(db)) | (np.abs(da - db) <= 1e-3)
    diff = ~same.all(axis=2)  # H x W
    H = diff.shape[0]
    return np.where(diff.any(axis=0), diff.argmax(axis=0), H)


def compare(tag, a, b, spp, full_rows=None):
    rgb_a, lin_a, gens_a = a
    rgb_b, lin_b, gens_b = b
    ok, eq, dmax = parity(lin_a, lin_b, rgb_a, rgb_b)
    H, W = lin_a.shape[:2]
    rows = first_diff_rows(lin_a, lin_b)
    diverged = int((rows < H).sum())
    # exposure: samples each column ran before diverging (a column diverging in row r ran >= r * spp
    # samples alike; counted at the row's start, which makes lam an upper estimate), censored at H * spp
    exposure = float(np.where(rows < H, rows * spp, H * spp).sum())
    lam = diverged / exposure if exposure > 0 else float("nan")
    out = {"cmp": tag, "W": W, "H": H, "spp": spp, "end_generators_equal": float((gens_a == gens_b).all(axis=1).mean()),
           "channels_within_1e-3": ok, "bytes_equal": eq, "max_abs_d": dmax, "columns_diverged": diverged,
           "divergence_per_sample": lam, "median_first_diff_row": float(np.median(rows))}
    if full_rows:  # predicted fraction of bit-identical pixels on a full frame of full_rows x spp_full
        fr, fs = full_rows
        r = np.arange(fr)
        out[f"predicted_identical_pixels_{fr}rows_{fs}spp"] = float(np.exp(-lam * (r + 1) * fs).mean())
        out[f"predicted_identical_columns_{fr}rows_{fs}spp"] = float(np.exp(-lam * fr * fs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--cam", default="cornell")
    ap.add_argument("--W", type=int, default=600)
    ap.add_argument("--H", type=int, default=600)
    ap.add_argument("--spp", type=int, default=1000)
    ap.add_argument("--rows", type=int, default=0, help="render only the top ROWS rows (tier A renders top down)")
    ap.add_argument("--full", type=str, default="", help="ROWSxSPP of the full frame to predict, e.g. 800x1000")
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--save", default="", help="write the oracle renders to this .npz")
    ap.add_argument("--load", default="", help="take the oracle renders from this .npz (written by --save)")
    a = ap.parse_args()
    earth = None
    if a.scene in ("earth", "random", "next_week_final"):
        earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"]
    sc, g1 = rtamd.make_scene(a.scene, rtamd.randGen(1024), earth=earth)
    # a crop of the top H' rows of the W x H frame: the full frame's camera with its lower-left corner
    # raised and its vertical span cut to H'/H (the same rays up to rounding), rendered as a W x H' frame
    # by every side (tier A's streams run top down, like the full frame's top rows)
    cam = rtamd.camera(a.cam, a.W, a.H)
    H = a.rows or a.H
    if H != a.H:
        f = H / a.H
        for i in range(3):
            cam.llc[i] = cam.llc[i] + cam.vert[i] * (1.0 - f)
            cam.vert[i] = cam.vert[i] * f
    gens = rtamd.column_gens(g1, a.W)
    full = tuple(int(x) for x in a.full.split("x")) if a.full else None
    res = {}
    t = {}
    saved = np.load(a.load) if a.load else None
    for name, flags in (("glibc", 0), ("rt_libm", rtamd.RT_FLAG_SHARED_LIBM)):
        if saved is not None:
            res[name] = tuple(saved[f"{name}_{k}"] for k in ("rgb", "lin", "gens"))
            t[f"oracle_{name}_s"] = float(saved[f"{name}_s"])
            continue
        p = rtamd.make_params(a.W, H, a.spp, 50, rtamd.RT_RNG_EXACT, flags=flags)
        t0 = time.time()
        rgb, lin, go, _ = pyoracle.render(sc, cam, p, col_gens=gens, nthreads=a.threads)
        t[f"oracle_{name}_s"] = time.time() - t0
        res[name] = (rgb, lin, go)
    if a.save:
        np.savez_compressed(a.save, **{f"{n}_{k}": v for n in ("glibc", "rt_libm")
                                       for k, v in zip(("rgb", "lin", "gens"), res[n])},
                            **{f"{n}_s": t[f"oracle_{n}_s"] for n in ("glibc", "rt_libm")})
    lines = [compare("oracle glibc vs oracle rt_libm.h (CPU proxy)", res["glibc"], res["rt_libm"], a.spp, full)]
    if a.gpu:
        # (a full-frame tier-A launch runs for minutes — one lane per column, every row and sample in
        # series: print a heartbeat so that the run is seen to be alive)
        import threading
        stop = threading.Event()

        def beat():
            t_start = time.time()
            while not stop.wait(30):
                print(f"  ... tier-A GPU render running, {time.time() - t_start:.0f} s", flush=True)
        threading.Thread(target=beat, daemon=True).start()
        ctx = rtamd.Context(0)
        ctx.upload(sc)
        for name, flags in (("ocml", 0), ("gpu_rt_libm", rtamd.RT_FLAG_SHARED_LIBM)):
            p = rtamd.make_params(a.W, H, a.spp, 50, rtamd.RT_RNG_EXACT, flags=flags)
            t0 = time.time()
            rgb, lin, go = ctx.render(cam, p, gens, linear=True, want_gens=True)
            t[f"gpu_{name}_s"] = time.time() - t0
            res[name] = (rgb, lin, go)
        ctx.close()
        stop.set()
        lines.append(compare("GPU OCML (runRenderAMD) vs oracle glibc", res["ocml"], res["glibc"], a.spp, full))
        same = compare("GPU rt_libm.h vs oracle rt_libm.h", res["gpu_rt_libm"], res["rt_libm"], a.spp)
        lines.append(same)
    for ln in lines:
        ln.update({"scene": a.scene, "frame": [a.W, a.H], "rows_rendered": H, "seconds": t})
        print(json.dumps(ln))
    if a.out:
        with open(a.out, "a") as f:
            for ln in lines:
                f.write(json.dumps(ln) + "\n")


if __name__ == "__main__":
    main()

"""Per-shard kernel time of a bench frame dealt over N ranks, measured on ONE GPU by rendering every
shard r of N in turn — an estimate of strong-scaling load balance and of the persistent kernel's tail,
without launching N processes. The N-GPU frame time is the slowest shard's.

    python scripts/shard_probe.py [--config c2] [--shards 1 2 4 8] [--reps 3] [--spp S]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing_amd"))
sys.path.insert(0, ROOT)

import rtamd  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--spp", type=int, default=0, help="override the config's spp (timing only)")
    a = ap.parse_args()
    import torch
    cfg = dict(CONFIGS[a.config])
    if a.spp:
        cfg["spp"] = a.spp
    earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"] if cfg.get("earth") else None
    scene, _ = rtamd.make_scene(cfg["scene"], rtamd.randGen(1024), param=cfg.get("param", 0), earth=earth)
    cam = rtamd.camera(cfg["camera"], cfg["W"], cfg["H"])
    ctx = rtamd.Context(0)
    ctx.upload(scene)
    out = {}
    for n in a.shards:
        times = []
        for r in range(n):  # every shard (the frame's time at N GPUs is the slowest one's)
            p = rtamd.make_params(cfg["W"], cfg["H"], cfg["spp"], cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024,
                                  tile=a.tile, shard_rank=r, shard_count=n)
            _, _, slab = rtamd.shard_geometry(p)
            buf = torch.zeros((slab, 3), dtype=torch.uint8, device="cuda")
            ms = []
            for _ in range(a.reps):
                ctx.render_shard_async(cam, p, buf.data_ptr())
                torch.cuda.synchronize()
                ms.append(ctx.last_kernel_ms())
            times.append(float(np.median(ms)))
        out[n] = {"max_shard_ms": round(max(times), 2), "mean_shard_ms": round(float(np.mean(times)), 2),
                  "min_shard_ms": round(min(times), 2), "shard_ms": [round(t, 2) for t in times]}
        print(json.dumps({"shards": n, **out[n]}), flush=True)
    base = out[a.shards[0]]["max_shard_ms"] * a.shards[0]
    for n in a.shards:
        print(f"N={n}: per-shard {out[n]['max_shard_ms']:.1f} ms (slowest of {n}; mean {out[n]['mean_shard_ms']:.1f}), "
              f"ideal {base / n:.1f} ms, efficiency {base / n / out[n]['max_shard_ms']:.3f}")
    ctx.close()


if __name__ == "__main__":
    main()

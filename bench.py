"""bench.py — MI355X throughput of the render path on BASELINE.json's headline configuration.

Metric (BASELINE.json): Msamples/s (W x H x spp / s) + achieved HBM GB/s on the In-One-Weekend
random scene (makeRandomSceneBookOne, src/Scenes.hs:253-317, randGen 1024), 1200x800, 500 spp,
depth 50. One step = one full frame rendered by the HIP kernel (tier B Philox streams), the
image tiles dealt round-robin over the N ranks, slabs all-gathered over RCCL and assembled on
rank 0. Scene and camera are resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1..c5] [--nan-cull]
        (N > 1: bench.py starts the N ranks itself, one process per GPU, RCCL world N)
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU; --gpus must equal N)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing_amd"))

import rtamd  # noqa: E402

# Config table. c2 is the headline; the others are reported on request.
CONFIGS = {
    "c1": dict(scene="three_spheres", camera="random_scene", W=200, H=100, spp=10, depth=10,
               desc="In-One-Weekend 3-sphere scene 200x100x10spp d10"),
    "c2": dict(scene="random_book_one", camera="random_scene", W=1200, H=800, spp=500, depth=50,
               desc="In-One-Weekend randomScene (makeRandomSceneBookOne) 1200x800x500spp d50"),
    "c3": dict(scene="cornell", camera="cornell", W=600, H=600, spp=1000, depth=50,
               desc="Cornell box (Rest-of-Your-Life) 600x600x1000spp d50"),
    "c4": dict(scene="next_week_final", camera="next_week", W=800, H=800, spp=1000, depth=50, earth=True,
               desc="The-Next-Week final scene (BVH, motion blur, Perlin, earthmap, media) 800x800x1000spp d50"),
    "c5": dict(scene="stress_spheres", camera="random_scene", W=3840, H=2160, spp=2000, depth=50, param=100000,
               desc="Stress: 100k random spheres 3840x2160x2000spp d50"),
}

# MI355X peaks (MI355X_MICROARCH.md chip table; FP64 vector = half the FP32 vector peak).
HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
FP32_PEAK_TFLOPS = 157.3

# Algorithmic bytes per unit of device-counted work (DESIGN.md "Roofline"): every BVH box test,
# leaf test and instance/medium test reads one 64-byte rt_node; every traced segment reads its
# hit material + texture (24 + 48 B); every light-pdf evaluation reads the light record (64 B);
# every pixel writes 3 bytes.
BYTES = {"box_tests": 64, "prim_tests": 64, "other_tests": 64, "segments": 72, "light_pdfs": 64,
         "wide_nodes": 128}  # a 4-wide node: four fp32 child boxes + four child ids (rt_wide.h)
# fp64 operations per unit (lower bound): box test 6 sub + 6 div + 6 min/max,
# sphere test ~30, scatter/shading ~60 per segment.
FLOPS = {"box_tests": 18, "prim_tests": 30, "other_tests": 30, "segments": 60}
# fp32 operations per 4-wide node: 4 children x (6 sub + 6 mul + 6 min/max + 3 for the test)
FLOPS32 = {"wide_nodes": 84}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(cfg, scene, cam, threads, spp_sample, budget_s=10.0):
    """The oracle (C restatement, tier-B streams) on a bounded sample of the same frame: samples
    0..spp-1 of every pixel of a band of rows around the middle of the image. A 1-spp probe of a
    thin band sizes the sample to about `budget_s` seconds (scenes differ ~100x in CPU cost per
    sample); `spp_sample` caps its spp. Also yields the per-sample work counters."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    W, H = cfg["W"], cfg["H"]

    def run(rows, spp):
        r0 = (H - rows) // 2
        p = rtamd.make_params(W, H, spp, cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024)
        t0 = time.perf_counter()
        _, _, _, cnt = pyoracle.render(scene, cam, p, rows=(r0, r0 + rows), nthreads=threads, linear=False,
                                       counters=True)
        return time.perf_counter() - t0, cnt, r0

    probe_rows = max(1, min(H, round(2e5 / W)))
    dt, _, _ = run(probe_rows, 1)
    rate = probe_rows * W / max(dt, 1e-6)  # samples/s
    n = rate * budget_s
    spp = int(max(1, min(spp_sample, n // (W * H))))
    rows = int(max(1, min(H, n // (W * spp))))
    dt, cnt, r0 = run(rows, spp)
    return rows * W * spp / dt / 1e6, dt, cnt, f"rows {r0}..{r0 + rows - 1} of {H} (all {W} columns) at {spp} spp"


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _latest_profile(suffix):
    """profiles/r<N>_<suffix> of the latest round that has one ('' when none)."""
    import glob
    import re
    best, path = -1, ""
    for f in glob.glob(os.path.join(ROOT, "profiles", f"r*_{suffix}")):
        m = re.match(r"r(\d+)_", os.path.basename(f))
        if m and int(m.group(1)) > best:
            best, path = int(m.group(1)), f
    return path


def default_selection(args):
    """True when this run launches the default kernel selection of its config (no RTAMD_* knobs, no
    culling / BVH / spp / tile overrides): only then does a committed PMC summary describe it."""
    return not any(k.startswith("RTAMD_") for k in os.environ) and not (
        args.nan_cull or args.reference_cull or args.reference_bvh or args.spp or args.tile != 8)


def _pmc_summary(args):
    path = args.traffic_json or _latest_profile(f"pmc_{args.config}.json")
    if not path or not os.path.exists(path) or not (default_selection(args) or args.traffic_json):
        return None, path
    with open(path) as f:
        return json.load(f), path


def pmc_traffic(args, kernel_ms, dispatches=1):
    """HBM traffic of the render kernel from the committed rocprofv3 PMC summary of the same
    config (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, bytes per dispatch), as GB/s over
    this run's live kernel time, and the bytes per frame step: a step of `dispatches` kernel launches
    (chunk batches, rt_launch_info.chunk_batches: C5 13) moves that many times the summary's
    per-dispatch bytes in its kernel time. None when no summary matches the launched kernel selection."""
    s, path = _pmc_summary(args)
    if s is None:
        return None, None, "no PMC summary for this kernel selection"
    b = s.get("derived", {}).get("hbm_bytes")
    if b is None:
        return None, None, f"{os.path.basename(path)} has no FETCH_SIZE/WRITE_SIZE"
    step = b * dispatches
    return round(step / (kernel_ms * 1e-3) / 1e9, 3), round(step), (
        f"{os.path.relpath(path, ROOT)}: {b / 1e6:.1f} MB per kernel dispatch HBM (FETCH_SIZE x2 + WRITE_SIZE) "
        f"x {dispatches} dispatch(es) per step, over the live kernel time; profiled dispatch "
        f"{s['avg_duration_s'] * 1e3:.1f} ms")


def pmc_valu(args):
    """The binding roof's view (VALU issue) from the same PMC summary: the share of the SIMDs'
    cycles the render kernel's vector instructions occupy, at 2 cycles per wave64 instruction on a
    SIMD-32 and 4 for fp64 ones (MI355X_MICROARCH.md: v_fma_f32 2 cycles; the fp64 vector peak is
    half the fp32 one), over the profiled launch's SIMD-cycles (1024 SIMDs x the measured clock),
    and the lane utilisation of the issued instructions. None unless the run launches the kernel
    selection the summary was profiled on (default_selection)."""
    s, path = _pmc_summary(args)
    if s is None:
        return None
    c, dur = s.get("counters_per_dispatch", {}), s.get("avg_duration_s")
    need = ("SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
            "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")
    if not dur or any(k not in c for k in need):
        return None
    f64 = sum(c[k] for k in need[2:])
    clock = c["GRBM_GUI_ACTIVE"] / 8 / dur  # GRBM_GUI_ACTIVE sums the 8 XCDs
    busy = (2 * (c["SQ_INSTS_VALU"] - f64) + 4 * f64) / (1024 * clock * dur)
    out = {"bound": "valu", "achieved": round(c["SQ_INSTS_VALU"] / dur / 1e9, 2),
           "peak": round(1024 * clock / 2 / 1e9, 2), "unit": "G wave-instr/s",
           "frac": round(busy, 4), "fp64_share": round(f64 / c["SQ_INSTS_VALU"], 4),
           "clock_ghz": round(clock / 1e9, 3),
           "lane_utilisation": round(s.get("derived", {}).get("valu_lane_utilisation", 0.0), 4),
           "kernels": s.get("kernels"), "profiled_launch_ms": round(dur * 1e3, 3),
           "source": os.path.relpath(path, ROOT),
           "note": "frac = SIMD cycles occupied by vector issue (2 per wave64 instruction, 4 per fp64 one) "
                   "over the profiled launch; achieved/peak count wave instructions at the 2-cycle rate"}
    return out


def sample_chunk(pixels, spp):
    """rt_sample_chunk (include/rt.h): samples per tier-B work-item."""
    fill = (pixels * spp + (1 << 20) - 1) >> 20
    ch = max(8, (spp + 127) // 128)
    ch = min(ch, spp, fill)
    return max(1, ch)


def algorithmic_offchip_bytes(cfg, p, scene):
    """Off-chip bytes the render kernel must move per launch, for this rank's slab: the chunk sums it
    writes (slab pixels x chunks x 24 B), the RGB8 slab combine_chunks writes (3 B per pixel), and the
    scene records read once (nodes incl. the device rebuild, 4-wide nodes, leaves, materials,
    textures, Perlin tables, image pool)."""
    _, _, slab = rtamd.shard_geometry(p)
    chunks = -(-cfg["spp"] // sample_chunk(cfg["W"] * cfg["H"], cfg["spp"]))
    d = scene.desc
    try:
        n_nodes = rtamd.rebuilt_scene(scene).desc.n_nodes
    except rtamd.RTError:
        n_nodes = d.n_nodes
    scene_b = (64 * n_nodes + 24 * d.n_materials + 48 * d.n_textures + 9216 * d.n_perlins + d.image_pool_bytes)
    out = {"chunk_sums": int(slab * chunks * 24), "image": int(slab * 3), "scene": int(scene_b)}
    out["total"] = sum(out.values())
    return out


def cpu_threads(args):
    """Threads for the CPU baseline: --cpu-threads if given, else the CPUs this process may run on
    (os.sched_getaffinity), capped by OMP_NUM_THREADS when the environment sets it (the GPU box
    sets it to this job's CPU share, 16 per GPU, while nproc shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    n = args.cpu_threads or min(aff, int(env) if env and env.isdigit() else aff)
    return n, {"affinity": aff, "nproc": os.cpu_count(), "omp_env": env}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_plan(gpus, env):
    """What this process is, from --gpus and its environment (no GPU touched):
    ("single", None) N = 1 and no launcher; ("rank", None) one rank of a launched world whose size
    matches --gpus; ("spawn", [env, ...]) N > 1 without a launcher: the per-rank environments of the N
    worker processes to start (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; one GPU per rank). Raises
    ValueError when a launcher's WORLD_SIZE disagrees with --gpus."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise ValueError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return ("rank" if world > 1 else "single"), None
    if gpus == 1:
        return "single", None
    port = env.get("MASTER_PORT") or str(_free_port())
    envs = []
    for r in range(gpus):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        envs.append(e)
    return "spawn", envs


def spawn_ranks(cmd, envs, poll_s=0.5):
    """Start one worker process per environment (the parent never touches the GPU), wait for all, and
    return the first non-zero exit code (0 when every rank succeeded). When a rank fails, the others
    are terminated (by their own PIDs) so that a barrier cannot hang the job."""
    import subprocess
    import threading
    # rank 0's stdout is filtered: its JSON line goes to stdout, anything else the runtime prints there
    # (gloo's connection notices) to stderr, so that stdout carries exactly one line; other ranks -> stderr
    # (ranks above 0 write to the parent's stderr descriptor; None (inherit) when sys.stderr has no
    # descriptor, e.g. under a capture wrapper)
    try:
        err_fd = sys.stderr.fileno()
    except (AttributeError, OSError, ValueError):
        err_fd = None
    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else err_fd, text=True)
             for r, e in enumerate(envs)]

    def forward(f):
        for line in f:
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()
    pump = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    pump.start()
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    log(f"[launcher] rank {procs.index(p)} exited with {code}; stopping the others")
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        pump.join(timeout=10)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--nan-cull", action="store_true", help="RT_FLAG_NAN_CULL (output-identical)")
    ap.add_argument("--reference-cull", action="store_true",
                    help="RT_FLAG_REFERENCE_CULL: the reference's per-axis box test only (no joint slab filter)")
    ap.add_argument("--reference-bvh", action="store_true",
                    help="traverse the reference's makeBVH world tree (default: SAH rebuild over the same leaves)")
    ap.add_argument("--spp", type=int, default=0, help="override spp (sampled runs of the big configs; not the metric)")
    ap.add_argument("--tile", type=int, default=8)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: the affinity CPU count, capped by OMP_NUM_THREADS)")
    ap.add_argument("--cpu-spp", type=int, default=0,
                    help="spp cap of the bounded CPU sample (default min(spp, 40M/(W*H)); a probe sizes the sample to ~10 s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-work", action="store_true", help="skip the counting-build pass")
    ap.add_argument("--traffic-json", default="",
                    help="PMC summary (scripts/pmc_summary.py) of this config's render kernel; default "
                         "profiles/r<latest>_pmc_<config>.json when the run uses the default kernel selection")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, default) or gloo (rehearsal: host-staged gather)")
    args = ap.parse_args()

    # --gpus N without a launcher: start N ranks (one process per GPU) before anything touches the GPU
    try:
        kind, envs = launch_plan(args.gpus, os.environ)
    except ValueError as e:
        log(f"bench.py: {e}")
        sys.exit(2)
    if kind == "spawn":
        log(f"[launcher] starting {args.gpus} ranks (backend {args.dist_backend}, port {envs[0]['MASTER_PORT']})")
        sys.exit(spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], envs))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev  # one process per GPU; a rehearsal may put several ranks on one device
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    cfg = dict(CONFIGS[args.config])
    if args.spp:
        cfg["spp"] = args.spp
        cfg["desc"] += f" [spp overridden to {args.spp}]"
    earth = None
    if cfg.get("earth"):
        earth = np.load(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"))["rgb"]
    scene, _ = rtamd.make_scene(cfg["scene"], rtamd.randGen(1024), param=cfg.get("param", 0), earth=earth)
    cam = rtamd.camera(cfg["camera"], cfg["W"], cfg["H"])
    ctx = rtamd.Context(local)
    ctx.upload(scene, reference_bvh=args.reference_bvh)
    flags = (rtamd.RT_FLAG_NAN_CULL if args.nan_cull else 0) | (
        rtamd.RT_FLAG_REFERENCE_CULL if args.reference_cull else 0)
    p = rtamd.make_params(cfg["W"], cfg["H"], cfg["spp"], cfg["depth"], rtamd.RT_RNG_PHILOX, seed=1024,
                          flags=flags, tile=args.tile, shard_rank=rank, shard_count=world)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    from rtamd.frame import ShardedFrame, device_assembler, device_renderer
    frame = ShardedFrame(p, world, rank, dev, args.dist_backend,
                         render=device_renderer(ctx, cam, stream.cuda_stream),
                         assemble=device_assembler(ctx, stream.cuda_stream))

    # device-measured work of this exact launch (counting build, outside the timed region)
    work = ctx.render_work(cam, p) if not args.no_work else None
    work_loop = ctx.last_launch()["loop"] if work else None  # (the counting build's walk: 2 = 4-wide, 1 = binary / mixed)

    for i in range(args.warmup):
        frame.step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup} done")
    frame.finish()
    frame.timings.clear()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        frame.step(kernel_ms=ctx.last_kernel_ms)  # (HIP events around the render launch, same stream)
        log(f"[rank {rank}] step {i + 1}/{args.steps}: kernel {frame._ev[-1][1]:.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    frame.finish()
    mine = frame.summary()  # this rank's mean kernel / all-gather / assemble ms
    per_rank = [mine]
    if world > 1:
        rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        kernel_avg = max(r["kernel_ms"] for r in per_rank)
    else:
        kernel_avg = mine["kernel_ms"]
    image = frame.image

    if rank == 0:
        samples_frame = cfg["W"] * cfg["H"] * cfg["spp"]
        value = samples_frame * args.steps / elapsed / 1e6
        ms_per_step = elapsed / args.steps * 1e3
        img = image.cpu().numpy()
        out = {
            "metric": "Msamples/s (WxHxspp/s) + achieved HBM GB/s, final scene 1200x800x500spp",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (scene generated by the reference's {cfg['scene']} builder from randGen 1024)",
            "config": {"workload": cfg["desc"], "width": cfg["W"], "height": cfg["H"], "spp": cfg["spp"],
                       "max_depth": cfg["depth"], "rng": "tier B Philox4x32-10 per (pixel, sample)",
                       "nan_cull": bool(args.nan_cull), "box_cull": "reference" if args.reference_cull else "joint",
                       "world_bvh": "reference makeBVH" if args.reference_bvh else "SAH rebuild (media-free worlds)",
                       "tile": args.tile, "parallelism": f"tiles x{world}"},
            "image_mean_rgb": [round(float(x), 3) for x in img.reshape(-1, 3).mean(0)],
        }
        cb = None
        counters = None
        if not args.no_cpu_baseline and world == 1:  # the CPU leg is timed at N=1 only
            if not args.cpu_spp:
                args.cpu_spp = max(1, min(cfg["spp"], round(40e6 / (cfg["W"] * cfg["H"]))))
            threads, cores = cpu_threads(args)
            v, dt, counters, what = cpu_baseline(cfg, scene, cam, threads, args.cpu_spp)
            cb = {"value": round(v, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
                  "affinity_cpus": cores["affinity"], "nproc": cores["nproc"],
                  "omp_num_threads_env": cores["omp_env"], "cpu": cpu_model(),
                  "sample": f"{what} (tier-B streams of the same frame), {dt:.1f} s, oracle/oracle.c fp64 glibc "
                            f"-O2 OpenMP, {threads} threads"}
        out["cpu_baseline"] = cb
        out["timing_per_rank_ms"] = [{k: round(v, 3) for k, v in r.items()} for r in per_rank]
        if world > 1:
            out["dist"] = {"backend": args.dist_backend, "world_size": dist.get_world_size(),
                           "slab_bytes_per_rank": int(frame.slab.numel()),
                           "note": "per rank: render kernel (HIP events), all-gather and assemble (events on the "
                                   "launch stream) means over the timed steps; assemble runs on rank 0 only"}
        if work:
            n = max(1, work["samples"])
            out["phase_split"] = {k: round(v, 4) for k, v in work.pop("phase_split").items()}
            slots = work.pop("lane_slots")
            leaf_hits, tie_redos = work.pop("leaf_hits"), work.pop("tie_redos")
            if slots["outer_iterations"]:  # lane utilisation of the replacement loop's phases
                out["lane_utilisation"] = {"shade": round(work["segments"] / slots["outer_iterations"], 4)}
                if work_loop == 2 and slots["wide_steps"] and slots["leaf_steps"]:  # (4-wide: two kinds of step)
                    out["lane_utilisation"]["wide_steps"] = round(work["wide_nodes"] / slots["wide_steps"], 4)
                    out["lane_utilisation"]["leaf_steps"] = round(work["prim_tests"] / slots["leaf_steps"], 4)
                elif slots["wide_steps"]:  # binary / mixed walk: node visits per lane slot of its steps, and how
                    # many node kinds (BVH box or 4-wide node, leaf primitive, instance, medium) one step runs
                    visits = work["box_tests"] + work["wide_nodes"] + work["prim_tests"] + work["other_tests"]
                    out["lane_utilisation"]["walk_steps"] = round(visits / slots["wide_steps"], 4)
                    out["walk_step_kinds"] = round(slots["leaf_steps"] / slots["wide_steps"], 4)
            per = {k: work[k] / n for k in work}
            bytes_per_sample = sum(BYTES[k] * per[k] for k in BYTES) + 3.0 / cfg["spp"]
            flops_per_sample = sum(FLOPS[k] * per[k] for k in FLOPS)
            f32 = sum(FLOPS32[k] * per.get(k, 0) for k in FLOPS32)
            samples_per_launch = samples_frame / world
            secs = kernel_avg * 1e-3
            fl = flops_per_sample * samples_per_launch / secs / 1e12
            fl32 = f32 * samples_per_launch / secs / 1e12
            # fp64-equivalent rate: an fp32 op costs half an fp64 one at the vector peaks (157.3 vs 78.6 TF)
            eq = fl + fl32 * FP64_PEAK_TFLOPS / FP32_PEAK_TFLOPS
            dispatches = max(1, int(ctx.last_launch().get("chunk_batches", 1)))
            traffic, tbytes, tnote = pmc_traffic(args, kernel_avg, dispatches)
            off = algorithmic_offchip_bytes(cfg, p, scene)
            out["roofline"] = {
                "bound": "fp64-valu", "achieved": round(eq, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(eq / FP64_PEAK_TFLOPS, 5),
                "traffic": traffic, "traffic_unit": "GB/s", "traffic_bytes_per_step": tbytes,
                "traffic_bytes_per_dispatch": round(tbytes / dispatches) if tbytes else None,
                "kernel_dispatches_per_step": dispatches,
                "algorithmic_offchip_bytes": off,
                "traffic_over_algorithmic": round(tbytes / off["total"], 3) if tbytes else None,
                "traffic_note": tnote,
                "kernel_ms": round(kernel_avg, 3),
                "flops_per_sample": {"fp64": round(flops_per_sample, 1), "fp32": round(f32, 1)},
                "note": "achieved = algorithmic fp64 flops per sample + fp32 flops at half weight (lower-bound "
                        "op counts per device-counted unit of work: box / leaf / instance tests, segments, "
                        "4-wide nodes; bench.py FLOPS), x samples per launch / the render kernel's HIP-event "
                        "time, against the fp64 vector peak: frac <= 1 by construction. The path is bound by "
                        "VALU issue under divergence and latency (valu_roofline: the PMC view), not by HBM: "
                        "traffic = PMC HBM bytes of the same kernel selection (FETCH_SIZE x2 + WRITE_SIZE) "
                        "next to the algorithmic off-chip bytes (chunk sums, image, scene records read once)"}
            out["scene_record_stream"] = {
                "bytes_per_sample": round(bytes_per_sample, 2),
                "gbs": round(bytes_per_sample * samples_per_launch / secs / 1e9, 2),
                "note": "algorithmic scene-record bytes per sample (4-wide nodes, leaves, materials) over the "
                        "kernel time: served from LDS and L2, so not an HBM figure"}
            out["valu_roofline"] = pmc_valu(args)
            out["fp64"] = {"achieved_tflops": round(fl, 3), "peak_tflops": FP64_PEAK_TFLOPS,
                           "frac": round(fl / FP64_PEAK_TFLOPS, 5), "flops_per_sample": round(flops_per_sample, 1)}
            out["fp32"] = {"achieved_tflops": round(fl32, 3), "peak_tflops": FP32_PEAK_TFLOPS,
                           "frac": round(fl32 / FP32_PEAK_TFLOPS, 5), "flops_per_sample": round(f32, 1)}
            out["work_per_sample"] = {k: round(v, 3) for k, v in per.items() if k != "samples"}
            out["work_per_sample"]["leaf_hits"] = round(leaf_hits / n, 3)
            out["work_per_sample"]["tie_redos"] = round(tie_redos / n, 5)
            if counters:
                out["work_per_sample_reference_cull"] = {k: round(v / max(1, counters["samples"]), 3)
                                                         for k, v in counters.items() if k != "samples"}
        else:
            out["roofline"] = None
        out["kernel_waves_per_simd"] = os.environ.get("RTAMD_WAVES", "default")
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

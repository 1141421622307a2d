"""Multi-rank tile sharding + gather on CPU (gloo, world size 2): each rank fills its slab from a
reference image through the shard map, slabs are all-gathered, and the assembled image must be
byte-identical to the reference. Mirrors bench.py's N>1 step (RCCL on the GPU box)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, tile, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ray-tracing_amd"))
    import torch
    import torch.distributed as dist
    import rtamd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img = np.random.default_rng(42).integers(0, 256, (H, W, 3), dtype=np.uint8)
    p = rtamd.make_params(W, H, 1, 1, tile=tile, shard_rank=rank, shard_count=world)
    m = rtamd.shard_pixel_map(p)
    slab = np.zeros((m.size, 3), dtype=np.uint8)
    slab[m >= 0] = img.reshape(-1, 3)[m[m >= 0]]
    t = torch.from_numpy(slab)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    if rank == 0:
        slabs = torch.stack(out).numpy()
        got = rtamd.assemble_host(slabs, p)
        q.put(bool(np.array_equal(got, img)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 120, 72, 16, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def _frame_worker(rank, world, port, W, H, tile, q, gather=None):
    """bench.py's step through rtamd.frame.ShardedFrame on the CPU: the renderer fills the rank's
    slab from a reference image through the shard map (as rt_render_shard_async lays it out), the
    slabs are all-gathered over gloo, rank 0 assembles with the assemble kernel's host restatement."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ray-tracing_amd"))
    import torch
    import torch.distributed as dist
    import rtamd
    from rtamd.frame import ShardedFrame, host_assembler
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img = np.random.default_rng(7).integers(0, 256, (H, W, 3), dtype=np.uint8)
    p = rtamd.make_params(W, H, 1, 1, tile=tile, shard_rank=rank, shard_count=world)
    calls = []

    def render(params, slab):
        m = rtamd.shard_pixel_map(params)
        s = np.zeros((m.size, 3), dtype=np.uint8)
        s[m >= 0] = img.reshape(-1, 3)[m[m >= 0]]
        slab.copy_(torch.from_numpy(s))
        calls.append(params.shard_rank)

    f = ShardedFrame(p, world, rank, "cpu", backend="gloo", render=render, assemble=host_assembler(), gather=gather)
    for _ in range(2):
        f.step()
    t = f.finish()
    ok = len(t) == 2 and calls == [rank, rank]
    if rank == 0:
        ok = ok and bool(np.array_equal(f.image.numpy(), img))
    q.put((rank, ok))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_sharded_frame_steps():
    """World size 3 (tiles dealt unevenly: 8 x 5 tiles over 3 ranks, padded slabs), two steps."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_frame_worker, args=(r, world, port, 120, 72, 16, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(res.values()), res


def test_gloo_sharded_frame_world_one_gathers():
    """gather=True at world size 1 runs the collective (the path the GPU suite runs over RCCL with a
    world-size-1 nccl group) and still assembles the image."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    proc = ctx.Process(target=_frame_worker, args=(0, 1, port, 97, 61, 16, q, True))
    proc.start()
    proc.join(120)
    assert proc.exitcode == 0
    assert q.get(timeout=5) == (0, True)

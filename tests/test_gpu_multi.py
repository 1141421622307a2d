"""The multi-GPU path on the GPU box: the C-ABI multi-device ctx (rt_create_multi: tile
shards rendered on every device from one host thread, gathered to the first with RCCL inside librtamd),
and bench.py's ShardedFrame over a torch nccl (= RCCL) process group. The one-GPU box has one device, so
both run RCCL at N = 1; N > 1 is the 8-GPU node's (the shard layout's invariance is covered by
test_gpu_parity.test_shard_invariance and the gloo tests)."""
import socket

import numpy as np
import pytest

import rtamd

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _device_lists():
    n = rtamd.device_count()
    return [[0]] + ([list(range(n))] if n > 1 else [])


@pytest.mark.parametrize("name,camname,w,h,spp", [("random_book_one", "random_scene", 160, 96, 8),
                                                  ("cornell_smoke", "cornell", 97, 61, 6)])
def test_multi_device_ctx_equals_one_device_render(gpu_ctx, name, camname, w, h, spp):
    """rt_render on a multi-device ctx (RCCL ncclGather of the slabs, assembled on the first device)
    gives the one-device render's bytes and linear averages, tier B; tier A renders on the first device
    (per-column streams do not shard) with the same bytes and end generators."""
    sc, g1 = rtamd.make_scene(name, rtamd.randGen(1024))
    cam = rtamd.camera(camname, w, h)
    p = rtamd.make_params(w, h, spp, 50, rtamd.RT_RNG_PHILOX, seed=5)
    pa = rtamd.make_params(w, h, 2, 50, rtamd.RT_RNG_EXACT)
    gens = rtamd.column_gens(g1, w)
    gpu_ctx.upload(sc)
    ref, lin_ref, _ = gpu_ctx.render(cam, p, linear=True)
    ref_a, _, gens_ref = gpu_ctx.render(cam, pa, gens, want_gens=True)
    for devs in _device_lists():
        m = rtamd.Context(devices=devs)
        try:
            assert m.devices() == devs
            m.upload(sc)
            allocs = []
            for _ in range(2):  # (two frames over the same communicators)
                rgb, lin, _ = m.render(cam, p, linear=True)
                assert np.array_equal(rgb, ref) and np.array_equal(lin, lin_ref, equal_nan=True)
                allocs.append(m.frame_timing()["device_allocs"])
            # the ctx keeps its slabs, gathered slabs, image and chunk sums: a second frame of the same size
            # allocates nothing on any device
            assert allocs[0] > 0 and allocs[1] == 0, allocs
            t = m.frame_timing()
            print(f"{name} on devices {devs}: kernel {['%.3f' % k for k in t['kernel_ms']]} ms, RCCL gather "
                  f"{t['gather_ms']:.3f} ms, assemble {t['assemble_ms']:.3f} ms, frame {t['frame_ms']:.3f} ms")
            assert t["n_devices"] == len(devs) and all(k > 0 for k in t["kernel_ms"])
            assert 0 < t["gather_ms"] < t["frame_ms"] and t["assemble_ms"] > 0
            rgb_a, _, gens_a = m.render(cam, pa, gens, want_gens=True)
            assert np.array_equal(rgb_a, ref_a) and np.array_equal(gens_a, gens_ref)
        finally:
            m.close()


def test_multi_device_ctx_full_c2_frame_costs_what_rt_render_costs(gpu_ctx):
    """The bench frame (C2: book one 1200x800x500, depth 50) through a one-device rt_create_multi ctx
    (slabs gathered by RCCL, assembled on device 0) against rt_render on a plain ctx: the same bytes, and
    the blocking call's wall time within 1 % (min of 3 frames each, legs alternating), with no device
    allocation after the first frame on either ctx."""
    import time
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 1200, 800)
    p = rtamd.make_params(1200, 800, 500, 50, rtamd.RT_RNG_PHILOX, seed=1024)
    gpu_ctx.upload(sc)
    m = rtamd.Context(devices=[0])
    try:
        m.upload(sc)
        ref, _, _ = gpu_ctx.render(cam, p)  # (warm-up frames: kernels loaded, buffers grown)
        got, _, _ = m.render(cam, p)
        assert np.array_equal(got, ref)
        wall = {"rt_render": [], "multi": []}
        for _ in range(3):
            for name, ctx in (("rt_render", gpu_ctx), ("multi", m)):
                t0 = time.perf_counter()
                ctx.render(cam, p)
                wall[name].append(time.perf_counter() - t0)
                assert ctx.frame_timing()["device_allocs"] == 0
        a, b = min(wall["rt_render"]), min(wall["multi"])
        t = m.frame_timing()
        print(f"C2 frame: rt_render {a * 1e3:.2f} ms, rt_create_multi(1) {b * 1e3:.2f} ms ({(b / a - 1) * 100:+.2f} %); "
              f"RCCL gather {t['gather_ms']:.3f} ms, assemble {t['assemble_ms']:.3f} ms")
        assert b <= 1.01 * a
    finally:
        m.close()


def test_multi_device_ctx_rejects_bad_lists():
    n = rtamd.device_count()
    for devs in ([0, 0], [n], [-1]):
        with pytest.raises(rtamd.RTError):
            rtamd.Context(devices=devs)


def test_multi_device_ctx_needs_a_scene_on_every_device():
    m = rtamd.Context(devices=[0])
    try:
        with pytest.raises(rtamd.RTError, match="no scene"):
            m.render(rtamd.camera("cornell", 16, 16), rtamd.make_params(16, 16, 1, 5))
    finally:
        m.close()


def test_sharded_frame_over_rccl_world_one(gpu_ctx):
    """bench.py's step (rtamd.frame.ShardedFrame) with gather=True in a world-size-1 nccl process group:
    init_process_group("nccl", device_id=...) and all_gather_into_tensor run on the box (RCCL) and the
    assembled frame equals rt_render's."""
    import torch
    import torch.distributed as dist

    from rtamd.frame import ShardedFrame, device_assembler, device_renderer
    sc, _ = rtamd.make_scene("random_book_one", rtamd.randGen(1024))
    cam = rtamd.camera("random_scene", 120, 80)
    gpu_ctx.upload(sc)
    p = rtamd.make_params(120, 80, 8, 50, rtamd.RT_RNG_PHILOX, seed=1024)
    ref, _, _ = gpu_ctx.render(cam, p)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        st = torch.cuda.current_stream(dev).cuda_stream
        f = ShardedFrame(p, 1, 0, dev, "nccl", render=device_renderer(gpu_ctx, cam, st),
                         assemble=device_assembler(gpu_ctx, st), gather=True)
        for _ in range(2):
            f.step(kernel_ms=gpu_ctx.last_kernel_ms)
        torch.cuda.synchronize()
        t = f.finish()
        print(f"ShardedFrame over RCCL, world 1: {t}")
        assert len(t) == 2 and all(x["gather_ms"] > 0 for x in t)
        assert np.array_equal(f.image.cpu().numpy(), ref)
    finally:
        dist.destroy_process_group()

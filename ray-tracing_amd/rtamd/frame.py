"""One frame of the multi-GPU render path: the step bench.py times.

The image is cut into tile x tile squares dealt round-robin over the ranks (rt_render_shard_async);
each rank renders its tiles into a slab, the slabs are all-gathered (RCCL over xGMI with the nccl
backend; host-staged with gloo), and rank 0 scatters them into the H x W x 3 image
(rt_assemble_async). The reference's only parallelism is row sparks (src/Lib.hs:1519-1520); tier-B
streams are per (pixel, sample), so the shards need no exchange before the final gather.

`ShardedFrame` is used by bench.py on the GPU and by the gloo tests on the CPU: the render and
assemble callables are injectable (`render(params, slab)`, `assemble(params, slabs, image)`), so the
CPU tests run the same gather / assemble / timing code as the bench.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np


class ShardedFrame:
    """Buffers and one step of a tile-sharded frame for `rank` of `world`.

    device: a torch device ("cuda:k" on the GPU box, "cpu" for gloo rehearsals and tests).
    backend: "nccl" (device all-gather) or "gloo" (host-staged all-gather).
    gather: run the all-gather through the process group (default: when world > 1). True at world 1
    exercises the collective path on one GPU (the slabs then round-trip through RCCL).
    """

    def __init__(self, params, world: int, rank: int, device, backend: str = "nccl",
                 render: Optional[Callable] = None, assemble: Optional[Callable] = None,
                 stream=None, gather: Optional[bool] = None):
        import torch

        import rtamd
        self.torch = torch
        self.p = params
        self.world, self.rank = world, rank
        self.device = torch.device(device)
        self.backend = backend
        self.cuda = self.device.type == "cuda"
        _, _, slab_px = rtamd.shard_geometry(params)
        self.slab = torch.zeros((slab_px, 3), dtype=torch.uint8, device=self.device)
        self.slabs = torch.zeros((world, slab_px, 3), dtype=torch.uint8, device=self.device)
        self.image = torch.zeros((params.height, params.width, 3), dtype=torch.uint8, device=self.device)
        self.stream = stream
        self._render = render
        self._assemble = assemble
        self.gather = world > 1 if gather is None else bool(gather)
        self.timings: List[dict] = []  # per step: kernel / all-gather / assemble (ms), filled by finish()
        self._ev: List[tuple] = []

    # ------------------------------------------------------------------ one step
    def step(self, kernel_ms: Optional[Callable[[], float]] = None):
        """Render this rank's slab, gather the slabs, assemble on rank 0 (stream-ordered on the GPU).

        Timings per step (finish()): GPU events after the render, after the collective, after the
        host-staged copy back to the device (gloo only) and after the assembly; and host wall-clock
        marks around the same phases, which add up to the step's wall time. (In a rehearsal whose
        ranks share one GPU the GPU intervals also hold the other ranks' kernels: e.g. rank 0's
        assembly queues behind rank 1's next render.)"""
        import time
        torch = self.torch
        h = [time.perf_counter()]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if self.cuda else None
        self._render(self.p, self.slab)
        if ev:
            ev[0].record()
        h.append(time.perf_counter())
        if self.gather:
            import torch.distributed as dist
            if self.backend == "nccl":
                dist.all_gather_into_tensor(self.slabs, self.slab)  # RCCL over xGMI
                if ev:
                    ev[1].record()
            else:
                host = self.slab.cpu()  # (waits for this rank's render)
                parts = [torch.empty_like(host) for _ in range(self.world)]
                dist.all_gather(parts, host)
                if ev:
                    ev[1].record()
                self.slabs.copy_(torch.stack(parts))  # the host-staged copy back to the device
            src = self.slabs
        else:
            src = self.slab
            if ev:
                ev[1].record()
        if ev:
            ev[2].record()
        h.append(time.perf_counter())
        if self.rank == 0:
            self._assemble(self.p, src, self.image)
        if ev:
            ev[3].record()
        h.append(time.perf_counter())
        self._ev.append((ev, kernel_ms() if kernel_ms else None, h))

    def finish(self) -> List[dict]:
        """Per-step timings (call after a device synchronize): render kernel ms (HIP events around
        the launch, from kernel_ms), all-gather, host-staged copy and assemble ms (events on the current
        stream), and the host wall-clock split of the step (host_*_ms)."""
        out = []
        for ev, kms, h in self._ev:
            t = {"kernel_ms": kms}
            if ev:
                t["gather_ms"] = ev[0].elapsed_time(ev[1])
                t["h2d_ms"] = ev[1].elapsed_time(ev[2])  # (gloo's host-staged copy; 0 with nccl)
                t["assemble_ms"] = ev[2].elapsed_time(ev[3])
            # host wall clock: enqueueing the render, the gather (gloo: waiting for the render, the
            # collective and the copy back), enqueueing the assembly
            t["host_render_ms"] = (h[1] - h[0]) * 1e3
            t["host_gather_ms"] = (h[2] - h[1]) * 1e3
            t["host_assemble_ms"] = (h[3] - h[2]) * 1e3
            out.append(t)
        self._ev.clear()
        self.timings.extend(out)
        return out

    def summary(self) -> dict:
        """Mean of each timing over the recorded steps."""
        keys = [k for k in ("kernel_ms", "gather_ms", "h2d_ms", "assemble_ms", "host_render_ms", "host_gather_ms",
                            "host_assemble_ms") if self.timings and self.timings[0].get(k) is not None]
        return {k: float(np.mean([t[k] for t in self.timings])) for k in keys}


def device_renderer(ctx, cam, stream_handle: int = 0):
    """render(params, slab) through rt_render_shard_async on the given HIP stream."""
    def render(p, slab):
        ctx.render_shard_async(cam, p, slab.data_ptr(), 0, stream_handle)
    return render


def device_assembler(ctx, stream_handle: int = 0):
    """assemble(params, slabs, image) through rt_assemble_async on the given HIP stream."""
    def assemble(p, slabs, image):
        ctx.assemble_async(p, slabs.data_ptr(), image.data_ptr(), stream_handle)
    return assemble


def host_assembler():
    """assemble(params, slabs, image) on the host (rtamd.assemble_host, the assemble kernel's
    restatement), for CPU rehearsals."""
    import rtamd

    def assemble(p, slabs, image):
        s = slabs if slabs.dim() == 3 else slabs.unsqueeze(0)
        image.copy_(image.new_tensor(rtamd.assemble_host(s.cpu().numpy(), p)))
    return assemble

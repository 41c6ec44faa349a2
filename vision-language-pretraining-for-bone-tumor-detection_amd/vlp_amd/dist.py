"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) / gloo on CPU.

Two exchanges per step:
  1. all-gather of the L2-normalised image/text embeddings ([B,E] each per rank)
     so every rank sees the global N x N contrastive matrix; the gradient of
     the gathered embeddings returns to the owners by reduce-scatter.
  2. SUM all-reduce of the flat per-tower gradient arenas (the global loss is
     a sum over ranks' row/column terms, so summed local gradients equal
     d L_global / d theta), in buckets launched while the backward is still
     running (GradReducer).  BatchNorm statistics stay per rank, as the
     reference's per-device BN (no SyncBN).

With the gloo backend (CPU tests, and the world-size-2 test of the real HIP
step that runs two ranks on one GPU) device tensors are staged through host
memory, since gloo has no reduce-scatter and no device transport: the
collectives are then synchronous and the result is copied back in place.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


# One-GPU rehearsal of the data-parallel schedule (bench.py --dp-rehearsal):
# with a world-1 process group initialised, every collective below is still
# issued (RCCL on one rank), and ClipStepFn wires the per-stage bucket
# callbacks exactly as at world > 1, so the multi-GPU stream schedule runs and
# is timed on one GPU.
REHEARSE = False


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def active() -> bool:
    """True when the step exchanges data: world > 1, or a world-1 group in rehearsal."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or REHEARSE


def _staged(t: torch.Tensor) -> bool:
    """gloo: no reduce-scatter, no device transport -> go through host memory."""
    return dist.get_backend() == "gloo"


class _Done:
    """Work handle of a collective that already completed (host-staged)."""

    def wait(self):
        return True


def all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    r, w = world()
    if not active():
        return x
    if _staged(x):
        parts = [torch.empty_like(x, device="cpu") for _ in range(w)]
        dist.all_gather(parts, x.detach().cpu().contiguous())
        return torch.cat(parts).to(x.device)
    out = torch.empty((w * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous())
    return out


def reduce_scatter_rows(x_all: torch.Tensor) -> torch.Tensor:
    r, w = world()
    if not active():
        return x_all
    rows = x_all.shape[0] // w
    if _staged(x_all):
        h = x_all.detach().to("cpu", copy=True).contiguous()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        return h[r * rows:(r + 1) * rows].to(x_all.device).contiguous()
    out = torch.empty((rows,) + tuple(x_all.shape[1:]), dtype=x_all.dtype, device=x_all.device)
    dist.reduce_scatter_tensor(out, x_all.contiguous(), op=dist.ReduceOp.SUM)
    return out


def all_reduce_sum_(t: torch.Tensor, async_op: bool = False):
    if not active():
        return None
    if _staged(t) and t.is_cuda:
        h = t.detach().cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        t.copy_(h)
        return _Done() if async_op else None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)


class GradReducer:
    """SUM all-reduce of flat gradient buffers, launched asynchronously as soon
    as each bucket is final and joined once at the end of the backward.

    `reduce(arenas)` launches one collective per arena (the head and text
    arenas: 0.1 / 57 MB); `reduce_span(arena, off, n)` one collective over a
    contiguous slice of an arena -- the image tower hands over its stages
    (layer4 -> stem, 52 / 27 / 4.5 / 0.9 MB) the moment their last weight
    gradient is folded, so all but the stem bucket overlap the rest of the
    backward (an RCCL collective runs on its own stream after the kernels
    already queued on the current one).  `wait()` joins them."""

    def __init__(self):
        self._work = []

    def reduce(self, arenas):
        for a in arenas:
            self.reduce_span(a, 0, a.grad.numel())

    def reduce_span(self, arena, off, n):
        if n <= 0:
            return
        w = all_reduce_sum_(arena.grad[off:off + n], async_op=True)
        if w is not None:
            self._work.append(w)

    def wait(self):
        for w in self._work:
            w.wait()
        self._work = []

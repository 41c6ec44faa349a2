"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) / gloo on CPU.

Two exchanges per step:
  1. all-gather of the L2-normalised image/text embeddings ([B,E] each per rank)
     so every rank sees the global N x N contrastive matrix; the gradient of
     the gathered embeddings returns to the owners by reduce-scatter.
  2. SUM all-reduce of the flat per-tower gradient arenas (the global loss is
     a sum over ranks' row/column terms, so summed local gradients equal
     d L_global / d theta).  BatchNorm statistics stay per rank, as the
     reference's per-device BN (no SyncBN).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    r, w = world()
    if w == 1:
        return x
    out = torch.empty((w * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous())
    return out


def reduce_scatter_rows(x_all: torch.Tensor) -> torch.Tensor:
    r, w = world()
    if w == 1:
        return x_all
    rows = x_all.shape[0] // w
    out = torch.empty((rows,) + tuple(x_all.shape[1:]), dtype=x_all.dtype, device=x_all.device)
    dist.reduce_scatter_tensor(out, x_all.contiguous(), op=dist.ReduceOp.SUM)
    return out


def all_reduce_sum_(t: torch.Tensor, async_op: bool = False):
    r, w = world()
    if w == 1:
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)


class GradReducer:
    """SUM all-reduce of flat gradient arenas.  `reduce(arenas)` launches one
    collective per arena (async), `wait()` joins them.  Arenas are large
    contiguous fp32 buffers (the image tower's is 85 MB), which is the bucket
    size xGMI ring/direct algorithms want."""

    def __init__(self):
        self._work = []

    def reduce(self, arenas):
        for a in arenas:
            w = all_reduce_sum_(a.grad, async_op=True)
            if w is not None:
                self._work.append(w)

    def wait(self):
        for w in self._work:
            w.wait()
        self._work = []

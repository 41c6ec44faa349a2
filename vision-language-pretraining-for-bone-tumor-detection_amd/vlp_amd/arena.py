"""Flat parameter arenas.

Every tower keeps its fp32 master parameters in ONE contiguous buffer (and its
gradients in a second one).  The named `nn.Parameter`s the state dict exposes
(timm / HF key names) are views into that buffer, so
  * the fused AdamW kernel updates a whole parameter group in one launch,
  * the data-parallel gradient all-reduce is one RCCL call per tower over a
    flat buffer (no bucketing copies),
  * bf16 operand copies of a whole tower are produced by one cast launch,
and checkpoints stay key-for-key compatible with the reference.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn as nn


class ParamArena:
    def __init__(self, specs: Sequence[Tuple[str, Tuple[int, ...]]], device=None, align: int = 64):
        self.layout: Dict[str, Tuple[int, int, Tuple[int, ...]]] = {}
        off = 0
        for name, shape in specs:
            n = 1
            for s in shape:
                n *= s
            self.layout[name] = (off, n, tuple(shape))
            off += (n + align - 1) // align * align  # 256-B aligned views
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)

    def view(self, name, buf=None):
        o, n, shape = self.layout[name]
        b = self.data if buf is None else buf
        return b[o:o + n].view(shape)

    def gview(self, name):
        return self.view(name, self.grad)

    def span(self, names: List[str]):
        """(offset, length) of the contiguous arena range covering `names`."""
        lo = min(self.layout[n][0] for n in names)
        hi = max(self.layout[n][0] + self.layout[n][1] for n in names)
        return lo, hi - lo


class ArenaModule(nn.Module):
    """A module whose parameters live in a ParamArena.

    `_apply` (used by .to()/.cuda()/.float()) is overridden so that device moves
    keep the parameters aliased to the arena."""

    def _init_arena(self, specs, device=None):
        self.arena = ParamArena(specs, device=device)
        self._param_slots: List[Tuple[nn.Module, str, str]] = []

    def _register(self, owner: nn.Module, attr: str, full_name: str):
        p = nn.Parameter(self.arena.view(full_name))
        owner.register_parameter(attr, p)
        self._param_slots.append((owner, attr, full_name))

    def _apply(self, fn, recurse=True):
        new_data = fn(self.arena.data)
        if new_data.dtype != torch.float32:
            raise TypeError("arena parameters are fp32 masters; cast the compute mode instead")
        self.arena.data = new_data
        self.arena.grad = fn(self.arena.grad)
        for owner, attr, full in self._param_slots:
            owner._parameters[attr].data = self.arena.view(full)
            owner._parameters[attr].grad = None
        for m in self.modules():
            for k, b in list(m._buffers.items()):
                if b is not None:
                    m._buffers[k] = fn(b)
        self._after_apply()
        return self

    def _after_apply(self):
        pass

    def params_in_arena_order(self):
        return [owner._parameters[attr] for owner, attr, _ in self._param_slots]

    @property
    def device(self):
        return self.arena.data.device

    def _aliased(self, p, full):
        return p.grad is not None and p.grad.data_ptr() == self.arena.gview(full).data_ptr()

    def begin_backward(self):
        """Call before a backward overwrites the grad arena.  After the first
        backward, p.grad IS a view of the arena (AccumulateGrad stole it); the
        backward then overwrites those values with the new gradient, and
        AccumulateGrad will add what grads_for_autograd returns to them.  So
        the values p.grad held before this backward (zeros after
        zero_grad(set_to_none=False), a running sum under gradient
        accumulation) are kept here and handed back instead of the gradient."""
        self._prior = None
        for owner, attr, full in self._param_slots:
            if self._aliased(owner._parameters[attr], full):
                self._prior = self.arena.grad.clone()
                return

    def grads_for_autograd(self, existing=None):
        """Per-parameter gradient tensors to hand back from an autograd
        Function, such that p.grad ends up = (its value before the backward)
        + (the new gradient written into the arena):
          p.grad None             -> the arena view (AccumulateGrad steals it)
          p.grad aliases the arena -> the pre-backward values (begin_backward)
          p.grad elsewhere        -> a copy of the new gradient."""
        prior = getattr(self, "_prior", None)
        out = []
        for owner, attr, full in self._param_slots:
            p = owner._parameters[attr]
            if not p.requires_grad:
                out.append(None)
                continue
            g = self.arena.gview(full)
            if p.grad is None:
                out.append(g)
            elif self._aliased(p, full):
                if prior is None:
                    raise RuntimeError("ArenaModule: begin_backward() was not called before this backward")
                out.append(self.arena.view(full, prior))
            else:
                out.append(g.clone())
        self._prior = None
        return out

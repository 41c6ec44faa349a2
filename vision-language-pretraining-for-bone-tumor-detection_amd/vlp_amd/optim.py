"""Fused AdamW over flat parameter arenas (replaces torch.optim.AdamW, the
reference's optimizer: configs/optimizer/adamw.yaml, built in
VisionLanguageModule.configure_optimizers :130-184 from the parameter groups of
_configure_optimizer_parameters :186-243).

Same parameter-group semantics as torch.optim.AdamW: per-group lr, parameters
whose .grad is None are skipped entirely (the unused TinyBERT pooler, as in the
reference), decoupled weight decay (torch default 0.01), bias correction with
the step count.  Each group is updated by one `vlp_adamw` launch per
contiguous arena span of parameters that have gradients.
"""
from __future__ import annotations

import torch

from . import ops


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 arenas=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        # map parameter -> (arena, offset, numel)
        self._loc = {}
        for a in arenas or []:
            mod = a
            for owner, attr, full in mod._param_slots:
                p = owner._parameters[attr]
                o, n, _ = mod.arena.layout[full]
                self._loc[id(p)] = (mod.arena, o, n)
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) not in self._loc:
                    raise ValueError("FusedAdamW: every parameter must live in a ParamArena")
        self._gstate = {}
        self._span_cache = {}

    def _spans(self, group):
        """Contiguous (arena, off, len) spans of params with gradients."""
        items = []
        for p in group["params"]:
            if p.grad is None:
                continue
            arena, o, n = self._loc[id(p)]
            g = arena.grad[o:o + n].view_as(p)
            if p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)  # gradients not produced in place (e.g. accumulated by autograd)
            items.append((arena, o, n))
        sig = tuple(t[1] for t in items) + tuple(id(t[0]) for t in items)
        cached = self._span_cache.get(sig)
        if cached is not None:
            return cached
        items.sort(key=lambda t: (id(t[0]), t[1]))
        spans = []
        for arena, o, n in items:
            if spans and spans[-1][0] is arena and self._gap_free(arena, spans[-1][1] + spans[-1][2], o):
                a, so, sn = spans[-1]
                spans[-1] = (a, so, o + n - so)
            else:
                spans.append((arena, o, n))
        self._span_cache[sig] = spans
        return spans

    @staticmethod
    def _gap_free(arena, end, start):
        """True if [end, start) holds only alignment padding (zeros with zero
        gradient, which AdamW leaves at zero), i.e. no other parameter."""
        if start < end:
            return False
        return not any(end <= o < start for o, _, _ in arena.layout.values())

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            st = self._gstate.setdefault(gi, {"step": 0, "m": {}, "v": {}})
            st["step"] += 1
            for arena, o, n in self._spans(group):
                key = (id(arena), o, n)
                if key not in st["m"]:
                    st["m"][key] = torch.zeros(n, dtype=torch.float32, device=arena.data.device)
                    st["v"][key] = torch.zeros(n, dtype=torch.float32, device=arena.data.device)
                ops.adamw(arena.data[o:o + n], arena.grad[o:o + n], st["m"][key], st["v"][key],
                          group["lr"], b1, b2, group["eps"], group["weight_decay"], st["step"])
        return loss

    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

"""Fused AdamW over flat parameter arenas (replaces torch.optim.AdamW, the
reference's optimizer: configs/optimizer/adamw.yaml, built in
VisionLanguageModule.configure_optimizers :130-184 from the parameter groups of
_configure_optimizer_parameters :186-243).

Same parameter-group semantics as torch.optim.AdamW: per-group lr, parameters
whose .grad is None are skipped entirely (the unused TinyBERT pooler, as in the
reference), decoupled weight decay (torch default 0.01), bias correction with
the parameter's step count.  Each group is updated by one `vlp_adamw` launch per
contiguous arena span of parameters that have gradients.

State: the first/second moments live in two flat fp32 buffers per arena (same
offsets as the parameters), and `self.state[p]` holds {"step", "exp_avg",
"exp_avg_sq"} with the moments as views of those buffers -- torch.optim.AdamW's
layout, so `state_dict()` / `load_state_dict()` round-trip (and a torch AdamW
state dict loads here) while the update stays one launch per span.
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
        self._flat = {}        # id(arena) -> (m, v) flat fp32 buffers
        self._span_cache = {}
        self._steps = {}       # id(p) -> step count (mirrored into state[p]["step"] by state_dict())

    def _moments(self, arena):
        b = self._flat.get(id(arena))
        if b is None or b[0].numel() != arena.numel or b[0].device != arena.data.device:
            b = (torch.zeros(arena.numel, dtype=torch.float32, device=arena.data.device),
                 torch.zeros(arena.numel, dtype=torch.float32, device=arena.data.device))
            self._flat[id(arena)] = b
        return b

    def _bind(self, p):
        """state[p] with moment views into the flat buffers (created at step 0)."""
        arena, o, n = self._loc[id(p)]
        m, v = self._moments(arena)
        st = self.state[p]
        mv, vv = m[o:o + n].view_as(p), v[o:o + n].view_as(p)
        if "exp_avg" in st and st["exp_avg"].data_ptr() != mv.data_ptr():
            mv.copy_(st["exp_avg"])       # loaded from a state dict: move into the flat buffer
            vv.copy_(st["exp_avg_sq"])
        st["exp_avg"], st["exp_avg_sq"] = mv, vv
        self._steps.setdefault(id(p), int(st["step"].item()) if "step" in st else 0)
        return st

    def _spans(self, group):
        """Contiguous (arena, off, len, [params]) spans of params with gradients."""
        items = []
        for p in group["params"]:
            if p.grad is None:
                continue
            arena, o, n = self._loc[id(p)]
            g = arena.grad[o:o + n].view_as(p)
            if p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)  # gradients not produced in place (e.g. accumulated by autograd)
            items.append((arena, o, n, p))
        sig = tuple(t[1] for t in items) + tuple(id(t[0]) for t in items)
        cached = self._span_cache.get(sig)
        if cached is not None:
            return cached
        items.sort(key=lambda t: (id(t[0]), t[1]))
        spans = []
        for arena, o, n, p in items:
            if spans and spans[-1][0] is arena and self._gap_free(arena, spans[-1][1] + spans[-1][2], o):
                a, so, sn, ps = spans[-1]
                spans[-1] = (a, so, o + n - so, ps + [p])
            else:
                spans.append((arena, o, n, [p]))
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
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for arena, o, n, ps in self._spans(group):
                steps = set()
                for p in ps:
                    if id(p) not in self._steps:
                        self._bind(p)
                    self._steps[id(p)] += 1
                    steps.add(self._steps[id(p)])
                if len(steps) != 1:
                    # parameters of one span disagree on their step count (a parameter
                    # that had no gradient in earlier steps): update them one by one
                    for p in ps:
                        _, po, pn = self._loc[id(p)]
                        self._launch(arena, po, pn, group, self._steps[id(p)])
                    continue
                self._launch(arena, o, n, group, steps.pop())
        return loss

    def _launch(self, arena, o, n, group, step):
        b1, b2 = group["betas"]
        m, v = self._moments(arena)
        ops.adamw(arena.data[o:o + n], arena.grad[o:o + n], m[o:o + n], v[o:o + n],
                  group["lr"], b1, b2, group["eps"], group["weight_decay"], step)

    def state_dict(self):
        for group in self.param_groups:
            for p in group["params"]:
                if id(p) in self._steps:
                    self.state[p]["step"] = torch.tensor(float(self._steps[id(p)]))
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._steps = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p in self.state and "exp_avg" in self.state[p]:
                    self.state[p]["step"] = torch.as_tensor(self.state[p]["step"], dtype=torch.float32).cpu()
                    self._bind(p)

    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

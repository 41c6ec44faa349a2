"""TinyBERT-4L-312D text tower on the HIP kernels (drop-in for
`AutoModel.from_pretrained("huawei-noah/TinyBERT_General_4L_312D")` wrapped by
TextEncoder, src/models/pretrain/VisionLanguageModule.py:38-60; the CLS hidden
state (token 0) is the sentence embedding, :52 / :60).

Parameter names are HF BertModel's (embeddings.*, encoder.layer.{i}.*,
pooler.dense.*), so `load_hf_state_dict` accepts a TinyBERT checkpoint as is.
The pooler exists (it is in the reference's optimizer) but, as in the
reference, receives no gradient.  Query/key/value weights are laid out
contiguously in the arena so one [936, 312] GEMM computes all three.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import ops
from .arena import ArenaModule


class TinyBertConfig:
    vocab_size = 30522
    hidden = 312
    layers = 4
    heads = 12
    ffn = 1200
    max_pos = 512
    type_vocab = 2
    ln_eps = 1e-12

    def __init__(self, hidden_dropout=0.1, attention_dropout=0.1):
        self.hidden_dropout = float(hidden_dropout)
        self.attention_dropout = float(attention_dropout)


class _Holder(nn.Module):
    pass


class TinyBertTower(ArenaModule):
    def __init__(self, config: TinyBertConfig = None, compute_dtype: str = "bf16", device=None):
        super().__init__()
        cfg = config or TinyBertConfig()
        self.cfg = cfg
        self.compute_dtype = compute_dtype
        D, F, L = cfg.hidden, cfg.ffn, cfg.layers
        specs = [("embeddings.word_embeddings.weight", (cfg.vocab_size, D)),
                 ("embeddings.position_embeddings.weight", (cfg.max_pos, D)),
                 ("embeddings.token_type_embeddings.weight", (cfg.type_vocab, D)),
                 ("embeddings.LayerNorm.weight", (D,)), ("embeddings.LayerNorm.bias", (D,))]
        for i in range(L):
            p = f"encoder.layer.{i}."
            # q/k/v weights then q/k/v biases: contiguous for the fused QKV GEMM
            specs += [(p + f"attention.self.{n}.weight", (D, D)) for n in ("query", "key", "value")]
            specs += [(p + f"attention.self.{n}.bias", (D,)) for n in ("query", "key", "value")]
            specs += [(p + "attention.output.dense.weight", (D, D)), (p + "attention.output.dense.bias", (D,)),
                      (p + "attention.output.LayerNorm.weight", (D,)), (p + "attention.output.LayerNorm.bias", (D,)),
                      (p + "intermediate.dense.weight", (F, D)), (p + "intermediate.dense.bias", (F,)),
                      (p + "output.dense.weight", (D, F)), (p + "output.dense.bias", (D,)),
                      (p + "output.LayerNorm.weight", (D,)), (p + "output.LayerNorm.bias", (D,))]
        specs += [("pooler.dense.weight", (D, D)), ("pooler.dense.bias", (D,))]
        # arena: no alignment padding inside the q/k/v groups (must be contiguous)
        self._init_arena_packed(specs, device)
        # module tree with HF names (registration order = HF state_dict order)
        emb = _Holder()
        self.embeddings = emb
        for n in ("word_embeddings", "position_embeddings", "token_type_embeddings"):
            h = _Holder()
            setattr(emb, n, h)
            self._register(h, "weight", f"embeddings.{n}.weight")
        ln = _Holder()
        emb.LayerNorm = ln
        self._register(ln, "weight", "embeddings.LayerNorm.weight")
        self._register(ln, "bias", "embeddings.LayerNorm.bias")
        enc = _Holder()
        self.encoder = enc
        enc.layer = nn.ModuleList()
        for i in range(L):
            p = f"encoder.layer.{i}."
            lay = _Holder()
            att = _Holder()
            lay.attention = att
            sa = _Holder()
            att.self = sa
            for n in ("query", "key", "value"):
                h = _Holder()
                setattr(sa, n, h)
                self._register(h, "weight", p + f"attention.self.{n}.weight")
                self._register(h, "bias", p + f"attention.self.{n}.bias")
            ao = _Holder()
            att.output = ao
            ao.dense = _Holder()
            self._register(ao.dense, "weight", p + "attention.output.dense.weight")
            self._register(ao.dense, "bias", p + "attention.output.dense.bias")
            ao.LayerNorm = _Holder()
            self._register(ao.LayerNorm, "weight", p + "attention.output.LayerNorm.weight")
            self._register(ao.LayerNorm, "bias", p + "attention.output.LayerNorm.bias")
            it = _Holder()
            lay.intermediate = it
            it.dense = _Holder()
            self._register(it.dense, "weight", p + "intermediate.dense.weight")
            self._register(it.dense, "bias", p + "intermediate.dense.bias")
            ou = _Holder()
            lay.output = ou
            ou.dense = _Holder()
            self._register(ou.dense, "weight", p + "output.dense.weight")
            self._register(ou.dense, "bias", p + "output.dense.bias")
            ou.LayerNorm = _Holder()
            self._register(ou.LayerNorm, "weight", p + "output.LayerNorm.weight")
            self._register(ou.LayerNorm, "bias", p + "output.LayerNorm.bias")
            enc.layer.append(lay)
        pool = _Holder()
        self.pooler = pool
        pool.dense = _Holder()
        self._register(pool.dense, "weight", "pooler.dense.weight")
        self._register(pool.dense, "bias", "pooler.dense.bias")
        self.reset_parameters()
        self._seed = 0x5EED
        self._ws = {}

    def _init_arena_packed(self, specs, device):
        from .arena import ParamArena
        self.arena = ParamArena(specs, device=device, align=1)
        self._param_slots = []

    @torch.no_grad()
    def reset_parameters(self):
        """HF BertPreTrainedModel._init_weights: N(0, 0.02) weights/embeddings,
        zero biases, LayerNorm 1/0."""
        for name, (o, n, shape) in self.arena.layout.items():
            v = self.arena.view(name)
            if "LayerNorm.weight" in name:
                v.fill_(1.0)
            elif name.endswith("bias"):
                v.zero_()
            else:
                v.normal_(0.0, 0.02)

    def _after_apply(self):
        self._ws = {}

    @property
    def tdtype(self):
        return torch.bfloat16 if self.compute_dtype == "bf16" else torch.float32

    def load_hf_state_dict(self, sd):
        """Load a HF BertModel state dict (e.g. TinyBERT_General_4L_312D)."""
        sd = {k[len("bert."):] if k.startswith("bert.") else k: v for k, v in sd.items()}
        return self.load_state_dict({k: v for k, v in sd.items() if k in self.state_dict()}, strict=False)

    def _wcopy(self):
        """Compute-dtype copy of the whole arena (one cast launch; same offsets)."""
        if self.compute_dtype == "fp32":
            return self.arena.data
        key = ("wT", str(self.arena.data.device))
        buf = self._ws.get(key)
        if buf is None:
            buf = torch.empty(self.arena.numel, dtype=self.tdtype, device=self.arena.data.device)
            self._ws[key] = buf
        ops.cast(self.arena.data, buf)
        return buf

    def _w(self, wT, name):
        return self.arena.view(name, wT)

    def _qkv(self, wT, i, bias=False, grad=False):
        p = f"encoder.layer.{i}.attention.self."
        names = [p + f"{n}.{'bias' if bias else 'weight'}" for n in ("query", "key", "value")]
        o, n = self.arena.span(names)
        D = self.cfg.hidden
        buf = self.arena.grad if grad else wT
        t = buf[o:o + n]
        return t if bias else t.view(3 * D, D)

    # ---------------- forward ----------------
    def run_forward(self, input_ids, attention_mask=None, token_type_ids=None, training=True, cls_only=False):
        """Returns (h, saved).  h = the last hidden state [B*T, D], or with
        cls_only the CLS rows only, [B, D]: the last encoder layer then runs its
        attention-output, LayerNorm and FFN work on the B CLS rows (its keys and
        values still cover every token), since the caller (VisionLanguageModule
        TextEncoder, :57-60) reads token 0 only."""
        cfg = self.cfg
        D, Fd, H = cfg.hidden, cfg.ffn, cfg.heads
        dh = D // H
        dev = self.arena.data.device
        T = self.tdtype
        B, Tn = input_ids.shape
        M = B * Tn
        ids = input_ids.contiguous().to(device=dev, dtype=torch.long)
        tt = None if token_type_ids is None else token_type_ids.contiguous().to(device=dev, dtype=torch.long)
        am = None if attention_mask is None else attention_mask.contiguous().to(device=dev, dtype=torch.long)
        wT = self._wcopy()
        A = self.arena.data
        p_h = cfg.hidden_dropout if training else 0.0
        p_a = cfg.attention_dropout if training else 0.0
        self._seed = (self._seed * 6364136223846793005 + 1442695040888963407) % (2 ** 63)
        seed = self._seed
        sv = {"B": B, "Tn": Tn, "ids": ids, "tt": tt, "seed": seed, "p_h": p_h, "p_a": p_a}
        e = torch.empty(M, D, dtype=T, device=dev)
        ops.embed_fwd(ids, tt, self.arena.view("embeddings.word_embeddings.weight"),
                      self.arena.view("embeddings.position_embeddings.weight"),
                      self.arena.view("embeddings.token_type_embeddings.weight"), e, M, Tn, D)
        h = torch.empty(M, D, dtype=T, device=dev)
        mu = torch.empty(M, device=dev)
        rs = torch.empty(M, device=dev)
        ops.layernorm_fwd(e, self.arena.view("embeddings.LayerNorm.weight"),
                          self.arena.view("embeddings.LayerNorm.bias"), cfg.ln_eps, h, mu, rs, M, D,
                          p=p_h, seed=seed + 1)
        sv["emb"] = (e, mu, rs)
        layers = []
        scale = 1.0 / math.sqrt(dh)
        for i in range(cfg.layers):
            p = f"encoder.layer.{i}."
            s_i = seed + 100 * (i + 1)
            if cls_only and i == cfg.layers - 1:
                layers.append(self._last_layer_cls(h, wT, A, am, B, Tn, p, s_i, p_h, p_a, scale))
                h = layers[-1]["h2"]
                break
            qkv = torch.empty(M, 3 * D, dtype=T, device=dev)
            ops.linear_fwd(h, self._qkv(wT, i), self._qkv(A, i, bias=True), qkv, M, 3 * D, D)
            ctx = torch.empty(M, D, dtype=T, device=dev)
            P = torch.empty(B, H, Tn, Tn, device=dev)
            ops.attn_fwd(qkv, am, ctx, P, B, Tn, H, dh, scale, p=p_a, seed=s_i + 1)
            s1 = torch.empty(M, D, dtype=T, device=dev)
            ops.linear_fwd(ctx, self._w(wT, p + "attention.output.dense.weight"),
                           self.arena.view(p + "attention.output.dense.bias"), s1, M, D, D, mode=2,
                           res=h, p=p_h, seed=s_i + 2)
            h1 = torch.empty(M, D, dtype=T, device=dev)
            mu1 = torch.empty(M, device=dev)
            rs1 = torch.empty(M, device=dev)
            ops.layernorm_fwd(s1, self.arena.view(p + "attention.output.LayerNorm.weight"),
                              self.arena.view(p + "attention.output.LayerNorm.bias"), cfg.ln_eps, h1,
                              mu1, rs1, M, D)
            u = torch.empty(M, Fd, dtype=T, device=dev)
            f = torch.empty(M, Fd, dtype=T, device=dev)
            ops.linear_fwd(h1, self._w(wT, p + "intermediate.dense.weight"),
                           self.arena.view(p + "intermediate.dense.bias"), f, M, Fd, D, mode=1, aux=u)
            s2 = torch.empty(M, D, dtype=T, device=dev)
            ops.linear_fwd(f, self._w(wT, p + "output.dense.weight"),
                           self.arena.view(p + "output.dense.bias"), s2, M, D, Fd, mode=2, res=h1,
                           p=p_h, seed=s_i + 3)
            h2 = torch.empty(M, D, dtype=T, device=dev)
            mu2 = torch.empty(M, device=dev)
            rs2 = torch.empty(M, device=dev)
            ops.layernorm_fwd(s2, self.arena.view(p + "output.LayerNorm.weight"),
                              self.arena.view(p + "output.LayerNorm.bias"), cfg.ln_eps, h2, mu2, rs2, M, D)
            layers.append({"h": h, "qkv": qkv, "ctx": ctx, "P": P, "s1": s1, "mu1": mu1, "rs1": rs1,
                           "h1": h1, "u": u, "f": f, "s2": s2, "mu2": mu2, "rs2": rs2, "seed": s_i})
            h = h2
        sv["layers"] = layers
        sv["wT"] = wT
        sv["h_last"] = h
        sv["cls_only"] = cls_only
        return h, sv

    def _last_layer_cls(self, h, wT, A, am, B, Tn, p, s_i, p_h, p_a, scale):
        """Last encoder layer for the CLS rows (row b*Tn of every [B*Tn] tensor,
        read in place through the GEMMs' leading dimensions)."""
        cfg = self.cfg
        D, Fd, H = cfg.hidden, cfg.ffn, cfg.heads
        dh = D // H
        M = B * Tn
        T, dev = self.tdtype, self.arena.data.device
        i = cfg.layers - 1
        qkv = torch.empty(M, 3 * D, dtype=T, device=dev)
        ops.linear_fwd(h, self._qkv(wT, i), self._qkv(A, i, bias=True), qkv, M, 3 * D, D)
        ctx = torch.empty(M, D, dtype=T, device=dev)
        P = torch.empty(B, H, Tn, Tn, device=dev)
        ops.attn_fwd(qkv, am, ctx, P, B, Tn, H, dh, scale, p=p_a, seed=s_i + 1)
        s1 = torch.empty(B, D, dtype=T, device=dev)
        ops.linear_fwd(ctx, self._w(wT, p + "attention.output.dense.weight"),
                       self.arena.view(p + "attention.output.dense.bias"), s1, B, D, D, ldx=Tn * D, mode=2,
                       res=h, ldr=Tn * D, p=p_h, seed=s_i + 2)
        h1 = torch.empty(B, D, dtype=T, device=dev)
        mu1 = torch.empty(B, device=dev)
        rs1 = torch.empty(B, device=dev)
        ops.layernorm_fwd(s1, self.arena.view(p + "attention.output.LayerNorm.weight"),
                          self.arena.view(p + "attention.output.LayerNorm.bias"), cfg.ln_eps, h1, mu1, rs1, B, D)
        u = torch.empty(B, Fd, dtype=T, device=dev)
        f = torch.empty(B, Fd, dtype=T, device=dev)
        ops.linear_fwd(h1, self._w(wT, p + "intermediate.dense.weight"),
                       self.arena.view(p + "intermediate.dense.bias"), f, B, Fd, D, mode=1, aux=u)
        s2 = torch.empty(B, D, dtype=T, device=dev)
        ops.linear_fwd(f, self._w(wT, p + "output.dense.weight"), self.arena.view(p + "output.dense.bias"), s2,
                       B, D, Fd, mode=2, res=h1, p=p_h, seed=s_i + 3)
        h2 = torch.empty(B, D, dtype=T, device=dev)
        mu2 = torch.empty(B, device=dev)
        rs2 = torch.empty(B, device=dev)
        ops.layernorm_fwd(s2, self.arena.view(p + "output.LayerNorm.weight"),
                          self.arena.view(p + "output.LayerNorm.bias"), cfg.ln_eps, h2, mu2, rs2, B, D)
        return {"h": h, "qkv": qkv, "ctx": ctx, "P": P, "s1": s1, "mu1": mu1, "rs1": rs1, "h1": h1, "u": u,
                "f": f, "s2": s2, "mu2": mu2, "rs2": rs2, "h2": h2, "seed": s_i, "cls": True}

    def _last_layer_cls_backward(self, Ls, dcls, wT, B, Tn, p_h, p_a, scale):
        """Backward of _last_layer_cls; returns the gradient of its input [B*Tn, D]."""
        cfg = self.cfg
        D, Fd, H = cfg.hidden, cfg.ffn, cfg.heads
        dh = D // H
        M = B * Tn
        T, dev = self.tdtype, self.arena.data.device
        G = self.arena
        i = cfg.layers - 1
        p = f"encoder.layer.{i}."
        s_i = Ls["seed"]
        dc = dcls.to(T).contiguous()
        ds2 = torch.empty(B, D, dtype=T, device=dev)
        dz = torch.empty(B, D, dtype=T, device=dev)
        ops.layernorm_bwd(dc, Ls["s2"], Ls["mu2"], Ls["rs2"], self.arena.view(p + "output.LayerNorm.weight"),
                          ds2, dz, G.gview(p + "output.LayerNorm.weight"), G.gview(p + "output.LayerNorm.bias"),
                          B, D, p_in=p_h, seed_in=s_i + 3)
        ops.colsum(dz, G.gview(p + "output.dense.bias"), B, D)
        ops.linear_wgrad(dz, Ls["f"], G.gview(p + "output.dense.weight"), B, D, Fd)
        du = torch.empty(B, Fd, dtype=T, device=dev)
        ops.linear_dgrad(dz, self._w(wT, p + "output.dense.weight"), du, B, Fd, D, mode=1, aux=Ls["u"])
        ops.colsum(du, G.gview(p + "intermediate.dense.bias"), B, Fd)
        ops.linear_wgrad(du, Ls["h1"], G.gview(p + "intermediate.dense.weight"), B, Fd, D)
        dh1 = torch.empty(B, D, dtype=T, device=dev)
        ops.linear_dgrad(du, self._w(wT, p + "intermediate.dense.weight"), dh1, B, D, Fd, addend=ds2)
        ds1 = torch.empty(B, D, dtype=T, device=dev)
        da = torch.empty(B, D, dtype=T, device=dev)
        ops.layernorm_bwd(dh1, Ls["s1"], Ls["mu1"], Ls["rs1"],
                          self.arena.view(p + "attention.output.LayerNorm.weight"), ds1, da,
                          G.gview(p + "attention.output.LayerNorm.weight"),
                          G.gview(p + "attention.output.LayerNorm.bias"), B, D, p_in=p_h, seed_in=s_i + 2)
        ops.colsum(da, G.gview(p + "attention.output.dense.bias"), B, D)
        ops.linear_wgrad(da, Ls["ctx"], G.gview(p + "attention.output.dense.weight"), B, D, D, ldx=Tn * D)
        # only the CLS queries receive a context gradient; the residual gradient
        # ds1 reaches the CLS rows of the layer input
        dctx = torch.zeros(M, D, dtype=T, device=dev)
        ops.linear_dgrad(da, self._w(wT, p + "attention.output.dense.weight"), dctx, B, D, D, lddx=Tn * D)
        dqkv = torch.empty(M, 3 * D, dtype=T, device=dev)
        ops.attn_bwd(Ls["qkv"], Ls["P"], dctx, dqkv, B, Tn, H, dh, scale, p=p_a, seed=s_i + 1)
        ops.colsum(dqkv, self._qkv(None, i, bias=True, grad=True), M, 3 * D)
        ops.linear_wgrad(dqkv, Ls["h"], self._qkv(None, i, grad=True), M, 3 * D, D)
        ds1_full = torch.zeros(M, D, dtype=T, device=dev)
        ops.scatter_rows(ds1, ds1_full, B, D, D, Tn * D)
        dh_new = torch.empty(M, D, dtype=T, device=dev)
        ops.linear_dgrad(dqkv, self._qkv(wT, i), dh_new, M, D, 3 * D, addend=ds1_full)
        return dh_new

    # ---------------- backward ----------------
    def run_backward(self, sv, dcls):
        """dcls: [B, D] gradient of the CLS hidden states (any dtype).  Zeroes and
        fills the grad arena (pooler gradient stays zero: unused, as in the reference)."""
        cfg = self.cfg
        D, Fd, H = cfg.hidden, cfg.ffn, cfg.heads
        dh = D // H
        dev = self.arena.data.device
        T = self.tdtype
        B, Tn = sv["B"], sv["Tn"]
        M = B * Tn
        wT = sv["wT"]
        G = self.arena
        G.grad.zero_()
        p_h, p_a = sv["p_h"], sv["p_a"]
        scale = 1.0 / math.sqrt(dh)
        top = cfg.layers - 1
        if sv.get("cls_only"):
            dh_ = self._last_layer_cls_backward(sv["layers"][top], dcls, wT, B, Tn, p_h, p_a, scale)
            top -= 1
        else:
            dh_ = torch.zeros(M, D, dtype=T, device=dev)
            dc = dcls.to(T).contiguous()
            ops.scatter_rows(dc, dh_, B, D, D, Tn * D)
        for i in range(top, -1, -1):
            p = f"encoder.layer.{i}."
            Ls = sv["layers"][i]
            s_i = Ls["seed"]
            # output LayerNorm: ds2 (residual) and dz = ds2 * dropout mask
            ds2 = torch.empty(M, D, dtype=T, device=dev)
            dz = torch.empty(M, D, dtype=T, device=dev)
            ops.layernorm_bwd(dh_, Ls["s2"], Ls["mu2"], Ls["rs2"], self.arena.view(p + "output.LayerNorm.weight"),
                              ds2, dz, G.gview(p + "output.LayerNorm.weight"), G.gview(p + "output.LayerNorm.bias"),
                              M, D, p_in=p_h, seed_in=s_i + 3)
            ops.colsum(dz, G.gview(p + "output.dense.bias"), M, D)
            ops.linear_wgrad(dz, Ls["f"], G.gview(p + "output.dense.weight"), M, D, Fd)
            du = torch.empty(M, Fd, dtype=T, device=dev)
            ops.linear_dgrad(dz, self._w(wT, p + "output.dense.weight"), du, M, Fd, D, mode=1, aux=Ls["u"])
            ops.colsum(du, G.gview(p + "intermediate.dense.bias"), M, Fd)
            ops.linear_wgrad(du, Ls["h1"], G.gview(p + "intermediate.dense.weight"), M, Fd, D)
            dh1 = torch.empty(M, D, dtype=T, device=dev)
            ops.linear_dgrad(du, self._w(wT, p + "intermediate.dense.weight"), dh1, M, D, Fd, addend=ds2)
            # attention output LayerNorm
            ds1 = torch.empty(M, D, dtype=T, device=dev)
            da = torch.empty(M, D, dtype=T, device=dev)
            ops.layernorm_bwd(dh1, Ls["s1"], Ls["mu1"], Ls["rs1"],
                              self.arena.view(p + "attention.output.LayerNorm.weight"), ds1, da,
                              G.gview(p + "attention.output.LayerNorm.weight"),
                              G.gview(p + "attention.output.LayerNorm.bias"), M, D, p_in=p_h, seed_in=s_i + 2)
            ops.colsum(da, G.gview(p + "attention.output.dense.bias"), M, D)
            ops.linear_wgrad(da, Ls["ctx"], G.gview(p + "attention.output.dense.weight"), M, D, D)
            dctx = torch.empty(M, D, dtype=T, device=dev)
            ops.linear_dgrad(da, self._w(wT, p + "attention.output.dense.weight"), dctx, M, D, D)
            dqkv = torch.empty(M, 3 * D, dtype=T, device=dev)
            ops.attn_bwd(Ls["qkv"], Ls["P"], dctx, dqkv, B, Tn, H, dh, scale, p=p_a, seed=s_i + 1)
            ops.colsum(dqkv, self._qkv(None, i, bias=True, grad=True), M, 3 * D)
            ops.linear_wgrad(dqkv, Ls["h"], self._qkv(None, i, grad=True), M, 3 * D, D)
            dh_new = torch.empty(M, D, dtype=T, device=dev)
            ops.linear_dgrad(dqkv, self._qkv(wT, i), dh_new, M, D, 3 * D, addend=ds1)
            dh_ = dh_new
        e, mu, rs = sv["emb"]
        de = torch.empty(M, D, dtype=T, device=dev)
        ops.layernorm_bwd(dh_, e, mu, rs, self.arena.view("embeddings.LayerNorm.weight"), de, None,
                          G.gview("embeddings.LayerNorm.weight"), G.gview("embeddings.LayerNorm.bias"),
                          M, D, p_out=p_h, seed_out=sv["seed"] + 1)
        ops.embed_bwd(sv["ids"], sv["tt"], de, G.gview("embeddings.word_embeddings.weight"),
                      G.gview("embeddings.position_embeddings.weight"),
                      G.gview("embeddings.token_type_embeddings.weight"), M, Tn, D)

    def grads_for_autograd(self, existing=None):
        out = super().grads_for_autograd()
        # pooler receives no gradient (only the CLS hidden state is used, :52/:60)
        for j, (owner, attr, full) in enumerate(self._param_slots):
            if full.startswith("pooler."):
                out[j] = None
        return out

    def forward(self, input_ids=None, attention_mask=None, token_type_ids=None, **kw):
        """API forward: returns the last hidden state [B, T, 312] (fp32) like
        BertModel(...).last_hidden_state."""
        return TextTowerFn.apply(self, input_ids, attention_mask, token_type_ids,
                                 *self.params_in_arena_order())


class TextTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tower, input_ids, attention_mask, token_type_ids, *params):
        h, sv = tower.run_forward(input_ids, attention_mask, token_type_ids, tower.training)
        ctx.tower, ctx.sv = tower, sv
        B, Tn = input_ids.shape
        return h.view(B, Tn, -1).float()

    @staticmethod
    def backward(ctx, dh):
        tower = ctx.tower
        B, Tn = ctx.sv["B"], ctx.sv["Tn"]
        # the API path gives a full [B,T,D] gradient; only CLS rows are non-zero in
        # the VLP model, but support the general case by scattering all rows
        dcls_rows = dh[:, 0, :].contiguous()
        if dh[:, 1:, :].abs().sum().item() != 0:  # pragma: no cover - generic last_hidden_state use
            raise NotImplementedError("TinyBertTower backward supports gradients on the CLS token only")
        tower.begin_backward()
        tower.run_backward(ctx.sv, dcls_rows)
        ctx.sv = None
        return (None, None, None, None, *tower.grads_for_autograd())

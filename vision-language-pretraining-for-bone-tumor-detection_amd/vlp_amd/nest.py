"""NesT image tower on the HIP kernels (drop-in for
`timm.create_model("nest_small", pretrained=False, num_classes=0, global_pool="avg", ...)`
behind ImageEncoder, src/models/pretrain/VisionLanguageModule.py:27-35;
SURVEY §8(f) row 2, BASELINE configs[3]: NesT-Small + TinyBERT at 512 x 512).

timm nest.py (timm==1.0.15) restated; parameter names are timm's, so a timm
checkpoint loads key for key (oracle/nest.py is the plain-torch restatement the
tests hold this tower to).  Per level (3 levels, dims 96 / 192 / 384, heads
3 / 6 / 12 of 32 channels, depths 2 / 2 / 20):
  level 0 input  = patch-embed GEMM (4x4/4 im2col written straight into the
                   level's blocked token order) + pos_embed
  level i > 0    = ConvPool (3x3 conv -> + bias -> LayerNorm(C) -> max pool
                   3x3/2) of the previous level's (deblockified) output,
                   blockified + pos_embed
  layer          = x + DropPath(proj(attn(qkv(LN1(x)))));  x + DropPath(fc2(GELU(fc1(LN2(x)))))
  head           = LayerNorm(384) over every token -> mean over tokens -> [B, 384]
Tokens stay in blocked order inside a level ([B][blocks][tokens][C] rows), so
the local attention of each block reads contiguous rows; the last level has a
single block, whose order is the image raster.  Attention runs the
flash-attention kernels of csrc/nest_ops.hip (head dim 32, scores never
stored); its head-major output meets the proj weight with its input columns
permuted from timm's (d*H + h) order once per step.

DropPath (stochastic depth, timm default drop_path_rate 0.5, rates linear in
depth): per-sample keep masks drawn on the host from the tower's own
generator each training step, uploaded with the step (`last_drop_masks`
exposes them so the tests replay the same masks in the oracle).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import ops
from .arena import ArenaModule

NEST_CFGS = {
    "nest_small": dict(embed_dims=(96, 192, 384), num_heads=(3, 6, 12), depths=(2, 2, 20)),
    "nest_tiny": dict(embed_dims=(96, 192, 384), num_heads=(3, 6, 12), depths=(2, 2, 8)),
    "nest_base": dict(embed_dims=(128, 256, 512), num_heads=(4, 8, 16), depths=(2, 2, 20)),
}
LN_EPS = 1e-6


class _Holder(nn.Module):
    pass


class NestTower(ArenaModule):
    def __init__(self, variant="nest_small", img_size=224, drop_rate=0.0, drop_path_rate=0.5,
                 compute_dtype="bf16", device=None, mlp_ratio=4.0, patch_size=4, num_levels=3):
        super().__init__()
        cfg = NEST_CFGS[variant]
        self.variant = variant
        self.img_size = int(img_size)
        self.dims, self.heads, self.depths = cfg["embed_dims"], cfg["num_heads"], cfg["depths"]
        if patch_size != 4 or num_levels != 3 or any(d // h != 32 for d, h in zip(self.dims, self.heads)):
            raise ValueError("NestTower: patch 4, 3 levels and 32-channel heads (every timm NesT variant)")
        self.mlp = [int(d * mlp_ratio) for d in self.dims]
        self.num_features = self.dims[-1]
        self.drop_rate = float(drop_rate)
        self.compute_dtype = compute_dtype
        grid = self.img_size // 4
        self.num_blocks = [4 ** i for i in range(num_levels)][::-1]           # 16, 4, 1
        if grid % 4:
            raise ValueError(f"NestTower: img_size {img_size} must give a patch grid divisible by 4")
        self.block_size = grid // 4
        self.seq = self.block_size ** 2
        dpr = torch.linspace(0, drop_path_rate, sum(self.depths)).tolist()
        self.dpr, k = [], 0
        for d in self.depths:
            self.dpr.append(dpr[k:k + d])
            k += d
        specs = [("patch_embed.proj.weight", (self.dims[0], 3, 4, 4)), ("patch_embed.proj.bias", (self.dims[0],))]
        for i, (C, F) in enumerate(zip(self.dims, self.mlp)):
            p = f"levels.{i}."
            specs.append((p + "pos_embed", (1, self.num_blocks[i], self.seq, C)))
            if i > 0:
                specs += [(p + "pool.conv.weight", (C, self.dims[i - 1], 3, 3)), (p + "pool.conv.bias", (C,)),
                          (p + "pool.norm.weight", (C,)), (p + "pool.norm.bias", (C,))]
            for j in range(self.depths[i]):
                q = p + f"transformer_encoder.{j}."
                specs += [(q + "norm1.weight", (C,)), (q + "norm1.bias", (C,)),
                          (q + "attn.qkv.weight", (3 * C, C)), (q + "attn.qkv.bias", (3 * C,)),
                          (q + "attn.proj.weight", (C, C)), (q + "attn.proj.bias", (C,)),
                          (q + "norm2.weight", (C,)), (q + "norm2.bias", (C,)),
                          (q + "mlp.fc1.weight", (F, C)), (q + "mlp.fc1.bias", (F,)),
                          (q + "mlp.fc2.weight", (C, F)), (q + "mlp.fc2.bias", (C,))]
        specs += [("norm.weight", (self.dims[-1],)), ("norm.bias", (self.dims[-1],))]
        self._init_arena(specs, device=device)
        # module tree with timm's names (registration order = timm state_dict order)
        for name, _ in specs:
            parts = name.split(".")
            owner = self
            for k, part in enumerate(parts[:-1]):
                if part.isdigit():
                    while len(owner) <= int(part):
                        owner.append(_Holder())
                    owner = owner[int(part)]
                    continue
                if part not in owner._modules:
                    setattr(owner, part, nn.ModuleList() if parts[k + 1].isdigit() else _Holder())
                owner = owner._modules[part]
            self._register(owner, parts[-1], name)
        self.reset_parameters()
        self._gen = torch.Generator().manual_seed(0x4E57)
        self.last_drop_masks = None
        self._ws = {}
        self.u8_norm = (127.5, 73.9)

    @torch.no_grad()
    def reset_parameters(self):
        """timm _init_nest_weights: Linear/Conv2d weights and pos_embed
        trunc_normal(std .02, a=-2, b=2), biases 0, LayerNorm 1 / 0."""
        for name, (o, n, shape) in self.arena.layout.items():
            v = self.arena.view(name)
            if name.endswith("pos_embed") or (name.endswith("weight") and len(shape) > 1):
                nn.init.trunc_normal_(v, std=0.02, a=-2, b=2)
            elif "norm" in name and name.endswith("weight"):
                v.fill_(1.0)
            else:
                v.zero_()

    def _after_apply(self):
        self._ws = {}

    @property
    def tdtype(self):
        return torch.bfloat16 if self.compute_dtype == "bf16" else torch.float32

    # ---------------- per-step weight copies ----------------
    def _weights(self):
        """Compute-dtype copy of the arena (one cast), the proj weights with
        their input columns in head-major order, and the packed conv weights."""
        dev, T = self.arena.data.device, self.tdtype
        ws = self._ws
        if "wT" not in ws:
            ws["wT"] = (self.arena.data if self.compute_dtype == "fp32"
                        else torch.empty(self.arena.numel, dtype=T, device=dev))
            ws["proj"] = {}
            ws["conv"] = {}
            for i, C in enumerate(self.dims):
                for j in range(self.depths[i]):
                    ws["proj"][(i, j)] = torch.empty(C, C, dtype=T, device=dev)
                if i > 0:
                    Ci = self.dims[i - 1]
                    ws["conv"][i] = (torch.empty(C, 3, 3, Ci, dtype=T, device=dev),
                                     torch.empty(Ci, 3, 3, C, dtype=T, device=dev))
        if self.compute_dtype != "fp32":
            ops.cast(self.arena.data, ws["wT"])
        for (i, j), wp in ws["proj"].items():
            C = self.dims[i]
            ops.nest_permute_cols(self.arena.view(f"levels.{i}.transformer_encoder.{j}.attn.proj.weight"), wp,
                                  C, self.heads[i], 32)
        for i, (wp, wt) in ws["conv"].items():
            ops.pack_conv(self.arena.view(f"levels.{i}.pool.conv.weight"), wp, wt)
        return ws

    def _w(self, wT, name):
        return self.arena.view(name, wT)

    def _drop_masks(self, B, training):
        """[level][layer] -> (attn scale, mlp scale) per sample, or None (no DropPath)."""
        if not training:
            self.last_drop_masks = None
            return None
        masks, host = [], []
        for i in range(3):
            lv = []
            for j in range(self.depths[i]):
                p = self.dpr[i][j]
                if p > 0.0:
                    m = torch.empty(2, B).bernoulli_(1 - p, generator=self._gen)
                    host.append(m / (1 - p))
                    lv.append((len(host) - 1, m))
                else:
                    lv.append(None)
            masks.append(lv)
        self.last_drop_masks = [[None if e is None else e[1] for e in lv] for lv in masks]
        if not host:
            return None
        dev = self.arena.data.device
        scales = torch.stack(host).to(dev, non_blocking=True)                  # [n][2][B]
        return [[None if e is None else (scales[e[0], 0], scales[e[0], 1]) for e in lv] for lv in masks]

    # ---------------- forward ----------------
    def run_forward(self, x, training, x_u8=None, u8_norm=None):
        """x: [B,3,H,W] fp32 (reference batch["x-ray"]) or x_u8 [B,1,H,W] uint8.
        Returns (features [B, 384] in the compute dtype, saved state)."""
        T, dev = self.tdtype, self.arena.data.device
        src = x if x is not None else x_u8
        B, Himg = src.shape[0], src.shape[-2]
        if Himg != self.img_size or src.shape[-1] != self.img_size:
            raise ValueError(f"NestTower: built for {self.img_size}x{self.img_size} inputs (timm img_size), "
                             f"got {tuple(src.shape[-2:])}")
        ws = self._weights()
        wT, A = ws["wT"], self.arena.data
        bs = self.block_size
        dpm = self._drop_masks(B, training)
        sv = {"B": B, "levels": [], "ws": ws, "dpm": dpm}
        # level 0 input: patch embedding straight into blocked token order, + pos_embed
        M0 = B * (self.img_size // 4) ** 2
        pm = torch.empty(M0, 48, dtype=T, device=dev)
        if x is not None:
            ops.nest_patch_prep(pm, B, Himg, Himg, bs, x=x.contiguous().float())
        else:
            mean, std = u8_norm if u8_norm is not None else self.u8_norm
            ops.nest_patch_prep(pm, B, Himg, Himg, bs, x_u8=x_u8.contiguous(), mean=mean, std=std)
        C0 = self.dims[0]
        h = torch.empty(M0, C0, dtype=T, device=dev)
        ops.linear_fwd(pm, self._w(wT, "patch_embed.proj.weight").view(C0, 48),
                       self.arena.view("patch_embed.proj.bias"), h, M0, C0, 48)
        ops.nest_add_bias(h, self.arena.view("levels.0.pos_embed").reshape(-1), B, self.num_blocks[0] * self.seq * C0)
        sv["pm"] = pm
        grid = self.img_size // 4
        for i, C in enumerate(self.dims):
            lv = {"C": C, "grid": grid}
            if i > 0:
                # ConvPool of the previous level's output image
                Ci = self.dims[i - 1]
                img = torch.empty(B, grid * 2, grid * 2, Ci, dtype=T, device=dev)
                g2 = grid * 2 // bs
                ops.nest_blockify(h, img, B, g2, g2, bs, Ci, inverse=True)
                wp, wt = ws["conv"][i]
                y = ops.conv_fwd(img, wp, C, 3, 3, 1, 1)
                Mi = B * (grid * 2) ** 2
                ops.nest_add_bias(y, self.arena.view(f"levels.{i}.pool.conv.bias"), Mi, C)
                z = torch.empty_like(y)
                mu = torch.empty(Mi, device=dev)
                rs = torch.empty(Mi, device=dev)
                ops.layernorm_fwd(y, self.arena.view(f"levels.{i}.pool.norm.weight"),
                                  self.arena.view(f"levels.{i}.pool.norm.bias"), LN_EPS, z, mu, rs, Mi, C)
                pooled = torch.empty(B, grid, grid, C, dtype=T, device=dev)
                idx = torch.empty(B, grid, grid, C, dtype=torch.uint8, device=dev)
                ops.nest_maxpool_fwd(z, pooled, idx)
                h = torch.empty(B * grid * grid, C, dtype=T, device=dev)
                g = grid // bs
                ops.nest_blockify(pooled, h, B, g, g, bs, C, pos=self.arena.view(f"levels.{i}.pos_embed"))
                lv["pool"] = {"img": img, "y": y, "mu": mu, "rs": rs, "idx": idx, "grid_in": grid * 2}
            lv["layers"] = []
            M = B * grid * grid
            H, F = self.heads[i], self.mlp[i]
            BT = B * self.num_blocks[i]
            for j in range(self.depths[i]):
                q = f"levels.{i}.transformer_encoder.{j}."
                L = {"x": h}
                y1 = torch.empty(M, C, dtype=T, device=dev)
                mu1, rs1 = torch.empty(M, device=dev), torch.empty(M, device=dev)
                ops.layernorm_fwd(h, self.arena.view(q + "norm1.weight"), self.arena.view(q + "norm1.bias"), LN_EPS,
                                  y1, mu1, rs1, M, C)
                qkv = torch.empty(M, 3 * C, dtype=T, device=dev)
                ops.linear_fwd(y1, self._w(wT, q + "attn.qkv.weight"), self.arena.view(q + "attn.qkv.bias"), qkv,
                               M, 3 * C, C)
                o = torch.empty(M, C, dtype=T, device=dev)
                lse = torch.empty(BT * H * self.seq, device=dev)
                ops.nest_attn_fwd(qkv, o, lse, BT, H, self.seq, 32 ** -0.5)
                dm = dpm[i][j] if dpm is not None else None
                x2 = self._residual(h, o, ws["proj"][(i, j)], self.arena.view(q + "attn.proj.bias"), M, C, C,
                                    dm[0] if dm is not None else None, B)
                y2 = torch.empty(M, C, dtype=T, device=dev)
                mu2, rs2 = torch.empty(M, device=dev), torch.empty(M, device=dev)
                ops.layernorm_fwd(x2, self.arena.view(q + "norm2.weight"), self.arena.view(q + "norm2.bias"), LN_EPS,
                                  y2, mu2, rs2, M, C)
                pre = torch.empty(M, F, dtype=T, device=dev)
                act = torch.empty(M, F, dtype=T, device=dev)
                ops.linear_fwd(y2, self._w(wT, q + "mlp.fc1.weight"), self.arena.view(q + "mlp.fc1.bias"), act, M, F,
                               C, mode=1, aux=pre)
                x3 = self._residual(x2, act, self._w(wT, q + "mlp.fc2.weight"), self.arena.view(q + "mlp.fc2.bias"),
                                    M, C, F, dm[1] if dm is not None else None, B)
                L.update(y1=y1, mu1=mu1, rs1=rs1, qkv=qkv, o=o, lse=lse, x2=x2, y2=y2, mu2=mu2, rs2=rs2, pre=pre,
                         act=act)
                lv["layers"].append(L)
                h = x3
            lv["out"] = h
            sv["levels"].append(lv)
            grid //= 2
        # head: LayerNorm over channels of every token, mean over tokens
        Cl = self.dims[-1]
        Ml = h.shape[0]
        zf = torch.empty(Ml, Cl, dtype=T, device=dev)
        muf, rsf = torch.empty(Ml, device=dev), torch.empty(Ml, device=dev)
        ops.layernorm_fwd(h, self.arena.view("norm.weight"), self.arena.view("norm.bias"), LN_EPS, zf, muf, rsf, Ml,
                          Cl)
        feat = torch.empty(B, Cl, dtype=T, device=dev)
        ops.avgpool_fwd(zf.view(B, Ml // B, 1, Cl), feat)
        sv["final"] = (h, muf, rsf, Ml // B)
        return feat, sv

    def _residual(self, x, a, w, bias, M, N, K, scale, B):
        """x + DropPath(a W^T + bias) (scale: per-sample 0 or 1/(1-p), None = identity)."""
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        if scale is None:
            ops.linear_fwd(a, w, bias, out, M, N, K, mode=2, res=x)
            return out
        ops.linear_fwd_rs(a, w, bias, out, x, scale, M // B, M, N, K)
        return out

    # ---------------- backward ----------------
    def run_backward(self, sv, dfeat, on_stage_done=None):
        """dfeat: [B, 384] gradient of the pooled features.  Overwrites the grad arena."""
        T, dev = self.tdtype, self.arena.data.device
        G = self.arena
        G.grad.zero_()
        ws = sv["ws"]
        wT = ws["wT"]
        B = sv["B"]
        bs = self.block_size
        dpm = sv["dpm"]
        h, muf, rsf, S = sv["final"]
        Cl = self.dims[-1]
        Ml = h.shape[0]
        dz = torch.empty(Ml, Cl, dtype=T, device=dev)
        ops.nest_bcast(dfeat.float().contiguous(), dz, B, S, Cl, 1.0 / S)
        dh = torch.empty(Ml, Cl, dtype=T, device=dev)
        ops.layernorm_bwd(dz, h, muf, rsf, self.arena.view("norm.weight"), dh, None, G.gview("norm.weight"),
                          G.gview("norm.bias"), Ml, Cl)
        for i in range(2, -1, -1):
            lv = sv["levels"][i]
            C, grid = lv["C"], lv["grid"]
            M = B * grid * grid
            H, F = self.heads[i], self.mlp[i]
            BT = B * self.num_blocks[i]
            dh_s = None
            for j in range(self.depths[i] - 1, -1, -1):
                q = f"levels.{i}.transformer_encoder.{j}."
                L = lv["layers"][j]
                dm = dpm[i][j] if dpm is not None else None
                # MLP branch (its DropPath-scaled gradient came out of the LN backward that
                # produced dh, except at a level's top layer)
                db = dh_s if dh_s is not None else self._branch_grad(dh, dm[1] if dm is not None else None, M, C, B)
                ops.colsum(db, G.gview(q + "mlp.fc2.bias"), M, C)
                ops.linear_wgrad(db, L["act"], G.gview(q + "mlp.fc2.weight"), M, C, F)
                dpre = torch.empty(M, F, dtype=T, device=dev)
                ops.linear_dgrad(db, self._w(wT, q + "mlp.fc2.weight"), dpre, M, F, C, mode=1, aux=L["pre"])
                ops.colsum(dpre, G.gview(q + "mlp.fc1.bias"), M, F)
                ops.linear_wgrad(dpre, L["y2"], G.gview(q + "mlp.fc1.weight"), M, F, C)
                dy2 = torch.empty(M, C, dtype=T, device=dev)
                ops.linear_dgrad(dpre, self._w(wT, q + "mlp.fc1.weight"), dy2, M, C, F)
                dx2 = torch.empty(M, C, dtype=T, device=dev)
                da = torch.empty(M, C, dtype=T, device=dev) if dm is not None else dx2
                ops.layernorm_bwd_add(dy2, L["x2"], L["mu2"], L["rs2"], self.arena.view(q + "norm2.weight"), dh, dx2,
                                      G.gview(q + "norm2.weight"), G.gview(q + "norm2.bias"), M, C,
                                      dxs=da if dm is not None else None, rscale=dm[0] if dm is not None else None,
                                      rps=M // B)
                # attention branch
                ops.colsum(da, G.gview(q + "attn.proj.bias"), M, C)
                dwp = self._proj_grad_ws(C)
                ops.linear_wgrad(da, L["o"], dwp, M, C, C)
                ops.nest_unpermute_cols(dwp, G.gview(q + "attn.proj.weight"), C, H, 32)
                do = torch.empty(M, C, dtype=T, device=dev)
                ops.linear_dgrad(da, ws["proj"][(i, j)], do, M, C, C)
                dqkv = torch.empty(M, 3 * C, dtype=T, device=dev)
                delta = torch.empty(BT * H * self.seq, device=dev)
                ops.nest_attn_bwd(L["qkv"], L["o"], do, L["lse"], delta, dqkv, BT, H, self.seq, 32 ** -0.5)
                ops.colsum(dqkv, G.gview(q + "attn.qkv.bias"), M, 3 * C)
                ops.linear_wgrad(dqkv, L["y1"], G.gview(q + "attn.qkv.weight"), M, 3 * C, C)
                dy1 = torch.empty(M, C, dtype=T, device=dev)
                ops.linear_dgrad(dqkv, self._w(wT, q + "attn.qkv.weight"), dy1, M, C, 3 * C)
                dx = torch.empty(M, C, dtype=T, device=dev)
                # the layer below's MLP-branch scale, applied in the same pass
                nm = dpm[i][j - 1] if (dpm is not None and j > 0) else None
                dh_s = torch.empty(M, C, dtype=T, device=dev) if nm is not None else None
                ops.layernorm_bwd_add(dy1, L["x"], L["mu1"], L["rs1"], self.arena.view(q + "norm1.weight"), dx2, dx,
                                      G.gview(q + "norm1.weight"), G.gview(q + "norm1.bias"), M, C,
                                      dxs=dh_s, rscale=nm[1] if nm is not None else None, rps=M // B)
                dh = dx
            # positional embedding: sum over the batch of the level-input gradient
            TN = self.num_blocks[i] * self.seq
            ops.nest_pos_grad(dh, G.gview(f"levels.{i}.pos_embed").view(TN, C), B, TN, C)
            if i == 0:
                # patch embedding (dh is in blocked order, as the patch rows)
                pm = sv["pm"]
                ops.colsum(dh, G.gview("patch_embed.proj.bias"), M, C)
                ops.linear_wgrad(dh, pm, G.gview("patch_embed.proj.weight").view(C, 48), M, C, 48)
                break
            # ConvPool backward: tokens -> pooled image grad -> max pool -> LN -> bias / conv
            P = lv["pool"]
            g = grid // bs
            dpool = torch.empty(B, grid, grid, C, dtype=T, device=dev)
            ops.nest_blockify(dh, dpool, B, g, g, bs, C, inverse=True)
            gi = P["grid_in"]
            dz = torch.empty(B, gi, gi, C, dtype=T, device=dev)
            ops.nest_maxpool_bwd(dpool, P["idx"], dz)
            Mi = B * gi * gi
            dyc = torch.empty_like(dz)
            ops.layernorm_bwd(dz, P["y"], P["mu"], P["rs"], self.arena.view(f"levels.{i}.pool.norm.weight"), dyc, None,
                              G.gview(f"levels.{i}.pool.norm.weight"), G.gview(f"levels.{i}.pool.norm.bias"), Mi, C)
            ops.colsum(dyc, G.gview(f"levels.{i}.pool.conv.bias"), Mi, C)
            Ci = self.dims[i - 1]
            ops.conv_wgrad_into(dyc, P["img"], 3, 3, 1, 1, G.gview(f"levels.{i}.pool.conv.weight"))
            wp, wt = ws["conv"][i]
            dimg = ops.conv_dgrad(dyc, wt, gi, gi, Ci, 3, 3, 1, 1)
            gp = gi // bs
            dh = torch.empty(B * gi * gi, Ci, dtype=T, device=dev)
            ops.nest_blockify(dimg, dh, B, gp, gp, bs, Ci)
        if on_stage_done is not None:
            on_stage_done(0, self.arena.numel)

    def _branch_grad(self, d, scale, M, C, B):
        if scale is None:
            return d
        out = torch.empty_like(d)
        ops.nest_rowscale(d, out, scale, M, C, M // B, 1)
        return out

    def _proj_grad_ws(self, C):
        buf = self._ws.get(("dproj", C))
        if buf is None:
            buf = torch.empty(C, C, device=self.arena.data.device)
            self._ws[("dproj", C)] = buf
        buf.zero_()
        return buf

    def stage_span(self, stage):
        return 0, self.arena.numel

    # ---------------- autograd entry ----------------
    def forward(self, x):
        """API forward: [B,3,H,W] float (or [B,1,H,W] uint8) -> [B, 384] fp32 features."""
        feat = NestTowerFn.apply(self, x, *self.params_in_arena_order())
        if self.drop_rate > 0.0 and self.training:
            feat = nn.functional.dropout(feat, self.drop_rate, True)
        return feat


class NestTowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tower: NestTower, x, *params):
        if x.dtype == torch.uint8:
            feat, saved = tower.run_forward(None, tower.training, x_u8=x, u8_norm=tower.u8_norm)
        else:
            feat, saved = tower.run_forward(x, tower.training)
        ctx.tower, ctx.saved = tower, saved
        return feat.float()

    @staticmethod
    def backward(ctx, dfeat):
        tower = ctx.tower
        tower.begin_backward()
        tower.run_backward(ctx.saved, dfeat.contiguous())
        ctx.saved = None
        return (None, None, *tower.grads_for_autograd())


def nest_flops_per_image(variant="nest_small", img_size=512):
    """Forward + backward FLOPs of one image (GEMMs, convs and attention; backward
    = 2x forward), for the bench's model-FLOP fraction."""
    cfg = NEST_CFGS[variant]
    grid = img_size // 4
    seq = (grid // 4) ** 2
    f = 2.0 * grid * grid * cfg["embed_dims"][0] * 48
    for i, (C, H, D) in enumerate(zip(cfg["embed_dims"], cfg["num_heads"], cfg["depths"])):
        tok = (grid >> i) ** 2
        if i > 0:
            f += 2.0 * (grid >> (i - 1)) ** 2 * C * cfg["embed_dims"][i - 1] * 9
        per = 2.0 * tok * (3 * C * C + C * C + 8 * C * C) + 4.0 * tok * seq * C
        f += D * per
    return 3.0 * f

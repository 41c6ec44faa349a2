"""ORACLE (test infrastructure): timm `nest_small` restated in plain torch.

Reference call site: src/models/pretrain/VisionLanguageModule.py:27-35
    timm.create_model(model, pretrained=False, num_classes=0, global_pool="avg", drop_rate=...)
with model = "nest_small" (the reference's baseline configs, e.g.
configs/experiment/baseline_only_imaging/baseline_only_imaging_nest_small.yaml:24;
BASELINE configs[3] pairs it with TinyBERT at 512x512, which needs img_size=512).
timm==1.0.15 (environment.yaml:327) is neither installed nor vendored, so this
restates its published nest.py -- PARITY UNPINNED against timm itself (no
reference test or fixture holds NesT outputs):

  Nest(img_size, in_chans=3, patch_size=4, num_levels=3, embed_dims=(96, 192, 384),
       num_heads=(3, 6, 12), depths=(2, 2, 20), mlp_ratio=4, qkv_bias=True,
       drop_path_rate=0.5, norm_layer=LayerNorm(eps=1e-6), act_layer=GELU)
  patch_embed.proj: Conv2d(3, 96, 4, 4)               -> [B, 96, H/4, W/4]
  levels.i (NestLevel): pool (ConvPool for i > 0: Conv2d(3x3, pad 1, bias) ->
      LayerNorm over channels -> MaxPool2d(3, 2, 1)), blockify into
      num_blocks = 4**(num_levels-1-i) blocks of block_size**2 tokens,
      + pos_embed [1, blocks, tokens, dim], transformer_encoder (pre-norm
      TransformerLayer: x + drop_path(attn(norm1(x))); x + drop_path(mlp(norm2(x)))),
      deblockify
  Attention: qkv Linear(dim, 3dim) -> (3, heads, dim/heads); softmax(q k^T / sqrt(d)) v;
      output permuted (B, T, N, d, heads) -> channel d*heads + h; proj Linear
  norm (LayerNorm over channels) -> global average pool -> [B, 384]
  init (timm _init_nest_weights): Linear / Conv2d weights trunc_normal(std .02,
      a=-2, b=2), biases 0; pos_embed trunc_normal(std .02); LayerNorm 1 / 0.
State-dict keys are timm's: patch_embed.proj.*, levels.{i}.pos_embed,
levels.{i}.pool.{conv,norm}.*, levels.{i}.transformer_encoder.{j}.{norm1,attn.qkv,
attn.proj,norm2,mlp.fc1,mlp.fc2}.*, norm.*.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

NEST_SMALL = dict(embed_dims=(96, 192, 384), num_heads=(3, 6, 12), depths=(2, 2, 20))


def blockify(x, block_size):
    B, H, W, C = x.shape
    gh, gw = H // block_size, W // block_size
    x = x.reshape(B, gh, block_size, gw, block_size, C)
    return x.transpose(2, 3).reshape(B, gh * gw, -1, C)


def deblockify(x, block_size):
    B, T, _, C = x.shape
    g = int(math.sqrt(T))
    x = x.reshape(B, g, g, block_size, block_size, C)
    return x.transpose(2, 3).reshape(B, g * block_size, g * block_size, C)


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, T, N, C = x.shape
        qkv = self.qkv(x).reshape(B, T, N, 3, self.num_heads, C // self.num_heads).permute(3, 0, 4, 1, 2, 5)
        q, k, v = qkv.unbind(0)
        attn = (q * self.scale) @ k.transpose(-2, -1)
        x = attn.softmax(dim=-1) @ v                                  # (B, H, T, N, d)
        x = x.permute(0, 2, 3, 4, 1).reshape(B, T, N, C)              # channel = d * H + h
        return self.proj(x)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


def drop_path(x, p, training, mask=None):
    """timm DropPath: per-sample keep mask / (1 - p); `mask` ([B] 0/1) overrides the RNG."""
    if p == 0.0 or not training:
        return x
    if mask is None:
        mask = torch.empty(x.shape[0], dtype=x.dtype).bernoulli_(1 - p)
    return x * (mask.to(x.dtype) / (1 - p)).view(-1, *([1] * (x.dim() - 1)))


class TransformerLayer(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio, drop_path):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.drop_path = drop_path
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.masks = None        # test hook: (attn mask, mlp mask) per sample

    def forward(self, x):
        m1, m2 = self.masks if self.masks is not None else (None, None)
        x = x + drop_path(self.attn(self.norm1(x)), self.drop_path, self.training, m1)
        return x + drop_path(self.mlp(self.norm2(x)), self.drop_path, self.training, m2)


class ConvPool(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 3, padding=1, bias=True)
        self.norm = nn.LayerNorm(cout, eps=1e-6)

    def forward(self, x):
        x = self.conv(x)
        x = self.norm(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return F.max_pool2d(x, 3, 2, 1)


class NestLevel(nn.Module):
    def __init__(self, num_blocks, block_size, seq_length, num_heads, depth, dim, prev_dim, mlp_ratio, dpr):
        super().__init__()
        self.block_size = block_size
        self.pos_embed = nn.Parameter(torch.zeros(1, num_blocks, seq_length, dim))
        self.pool = ConvPool(prev_dim, dim) if prev_dim is not None else nn.Identity()
        self.transformer_encoder = nn.Sequential(*[TransformerLayer(dim, num_heads, mlp_ratio, dpr[i])
                                                   for i in range(depth)])

    def forward(self, x):
        x = self.pool(x).permute(0, 2, 3, 1)
        x = blockify(x, self.block_size) + self.pos_embed
        x = self.transformer_encoder(x)
        return deblockify(x, self.block_size).permute(0, 3, 1, 2)


class Nest(nn.Module):
    def __init__(self, img_size=224, in_chans=3, patch_size=4, num_levels=3, embed_dims=(96, 192, 384),
                 num_heads=(3, 6, 12), depths=(2, 2, 20), mlp_ratio=4.0, drop_rate=0.0, drop_path_rate=0.5):
        super().__init__()
        self.num_features = embed_dims[-1]
        self.drop_rate = drop_rate
        num_blocks = [4 ** i for i in range(num_levels)][::-1]
        grid = img_size // patch_size
        assert grid % int(math.sqrt(num_blocks[0])) == 0
        self.block_size = grid // int(math.sqrt(num_blocks[0]))
        seq_length = grid * grid // num_blocks[0]
        self.patch_embed = nn.Module()
        self.patch_embed.proj = nn.Conv2d(in_chans, embed_dims[0], patch_size, patch_size)
        dprs = torch.linspace(0, drop_path_rate, sum(depths)).split(list(depths))
        levels, prev = [], None
        for i in range(num_levels):
            levels.append(NestLevel(num_blocks[i], self.block_size, seq_length, num_heads[i], depths[i],
                                    embed_dims[i], prev, mlp_ratio, [float(v) for v in dprs[i]]))
            prev = embed_dims[i]
        self.levels = nn.Sequential(*levels)
        self.norm = nn.LayerNorm(embed_dims[-1], eps=1e-6)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        for lvl in self.levels:
            nn.init.trunc_normal_(lvl.pos_embed, std=0.02, a=-2, b=2)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.trunc_normal_(m.weight, std=0.02, a=-2, b=2)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward_features(self, x):
        x = self.patch_embed.proj(x)
        x = self.levels(x)
        return self.norm(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)

    def forward(self, x):
        x = self.forward_features(x).mean((2, 3))
        return F.dropout(x, self.drop_rate, self.training) if self.drop_rate > 0 else x


def nest_small(img_size=224, **kw):
    return Nest(img_size=img_size, **{**NEST_SMALL, **kw})

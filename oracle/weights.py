"""ORACLE (test infrastructure): deterministic, name-keyed weight recipe.

The reference's encoders start from timm init (conv kaiming, zero bn2 gamma) and
TinyBERT hub weights (unavailable offline).  Parity runs instead fill every
parameter/buffer from a generator seeded by (seed, crc32(name)), so the golden
generator (which runs the reference code), the CPU oracle and the HIP model
all hold bit-identical fp32 weights without shipping 143 MB of fixtures.
bn2 gammas are non-zero so every residual branch carries gradient.
"""
import math
import zlib

import torch


def _gen(name: str, seed: int) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((seed * 1000003 + zlib.crc32(name.encode())) % (2 ** 63))
    return g


def value_for(name: str, shape, seed: int = 0) -> torch.Tensor:
    g = _gen(name, seed)
    shape = tuple(shape)
    last = name.rsplit(".", 1)[-1]
    if name.endswith("num_batches_tracked"):
        return torch.zeros(shape, dtype=torch.long)
    if name == "logit_scale":
        return torch.full(shape, math.log(1 / 0.07))
    if name in ("image_projection", "text_projection"):
        return torch.randn(shape, generator=g, dtype=torch.float64).float() * shape[0] ** -0.5
    is_bn = (".bn" in name or "downsample.1" in name) and name.startswith("image_encoder")
    is_ln = "LayerNorm" in name
    if is_bn or is_ln:
        if last == "weight":
            return (torch.rand(shape, generator=g, dtype=torch.float64) * 0.8 + 0.6).float()
        if last == "bias":
            return (torch.randn(shape, generator=g, dtype=torch.float64) * 0.1).float()
        if last == "running_mean":
            return (torch.randn(shape, generator=g, dtype=torch.float64) * 0.1).float()
        if last == "running_var":
            return (torch.rand(shape, generator=g, dtype=torch.float64) * 0.8 + 0.6).float()
    if len(shape) == 4:  # conv, kaiming fan_out
        fan_out = shape[0] * shape[2] * shape[3]
        return (torch.randn(shape, generator=g, dtype=torch.float64) * math.sqrt(2.0 / fan_out)).float()
    if "embeddings" in name:
        return (torch.randn(shape, generator=g, dtype=torch.float64) * 0.05).float()
    if len(shape) == 2:  # linear weight [out][in]
        return (torch.randn(shape, generator=g, dtype=torch.float64) * shape[1] ** -0.5).float()
    if last == "bias":
        return (torch.randn(shape, generator=g, dtype=torch.float64) * 0.02).float()
    raise KeyError(f"no recipe for {name} {shape}")


def recipe_state_dict(named_shapes, seed: int = 0):
    """named_shapes: iterable of (name, shape) -> {name: tensor}"""
    return {n: value_for(n, s, seed) for n, s in named_shapes}


def apply_recipe(module: torch.nn.Module, seed: int = 0):
    sd = module.state_dict()
    new = {k: value_for(k, v.shape, seed).to(v.dtype) for k, v in sd.items()}
    module.load_state_dict(new)
    return module

"""The bf16 throughput path at the benchmark configuration (BASELINE configs[1]:
bs = 256, 512 x 512, T = 40) against the fp32 CPU oracle on the same weights
and the same batch.

This is the engine the bench measures: the LDS-DMA big-tile GEMMs, the W = 128
layer-1 rows kernel, the full-size stem and maxpool, the bf16 text tower --
none of which run in the fp32 parity-mode tests.  Weights: the module's own
initialisation, as the bench and the reference start training (timm resnet34
init with zero-initialised last BN of each block, HF BERT init); one train-mode
step (batch-statistics BN, text dropout off) on each side.  The oracle's fp32
forward + backward of the 256-pair batch takes ~45-60 s on 16 host cores.

What bf16 can reach: the gradients of a bf16 step differ from fp32 by 10-20 %
on this model, for any bf16 implementation -- bf16 rounding of the embeddings
(~5e-3) is multiplied by the logit scale exp(logit_scale) = 14.3 in the softmax,
and the BN backward amplifies the deviation of the feature gradient.  PyTorch's
own bf16 autocast shows it (tools: the autocast test below measures it at a
small shape on the CPU): the HIP bf16 step must be at least as close to fp32 as
torch's bf16 autocast is, per gradient group.

Gates (measured values are printed):
  bs=256: loss |delta| <= 5e-2 (measured ~3e-6..3e-3), probe
    features (eval, first 32 images) and embeddings rel-L2 <= 2e-2; gradient
    groups vs fp32 (whole image-tower conv vector, BN params, projections,
    text tower) <= 0.30 (measured 0.06-0.23)
    and per tensor <= 0.4 (BN parameters, sums of cancelling terms: 0.8), median <= 0.1
  bs=16, 256 px: every group's error <= 1.5 x torch-autocast-bf16's + 0.01, every
    tensor's <= 1.5 x torch autocast's own error on that tensor + 0.02
"""
import functools
import statistics

import pytest
import torch

from oracle.clip import OracleVLP, compute_loss
from tests.golden.synth import synth_batch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def cosine(a, b):
    a, b = a.double().flatten().cpu(), b.double().flatten().cpu()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def module_init_state():
    """The module's own init (what bench.py and a fresh training run start from)."""
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    torch.manual_seed(0)
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    del m
    return sd


def hip_bf16(sd, batch, probe=None):
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="bf16", text_dropout=0.0)
    m.load_state_dict(sd)
    feats = None
    if probe is not None:
        m.eval()
        with torch.no_grad():
            feats = m.image_encoder(probe.cuda()).float().cpu()
    m.train()
    loss, li, lt, ie, te = m.training_step_outputs(batch)
    loss.backward()
    torch.cuda.synchronize()
    out = {"loss": loss.item(), "ie": ie.float().cpu(), "te": te.float().cpu(), "feats": feats,
           "grads": {k: p.grad.float().cpu() for k, p in m.named_parameters() if p.grad is not None}}
    del m
    torch.cuda.empty_cache()
    return out


def cpu_oracle(sd, batch, probe=None, autocast=False):
    o = OracleVLP(128, text_dropout=0.0)
    o.load_state_dict(sd)
    feats = None
    if probe is not None:
        o.eval()
        with torch.no_grad():
            feats = o.image_encoder(probe)
    o.train()
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
        lg, ie, te = o(batch)
    lo = compute_loss(lg.float())[0]
    lo.backward()
    return {"loss": lo.item(), "ie": ie.detach().float(), "te": te.detach().float(), "feats": feats,
            "grads": {k: p.grad.float() for k, p in o.named_parameters() if p.grad is not None}}


def group_errors(ga, gb):
    """rel-L2 per gradient group (parameters with an exactly-zero fp32 gradient --
    the residual branches behind a zero-initialised BN, the attention key biases --
    carry no signal and are left out)."""
    keys = [k for k in gb if k in ga and gb[k].norm() > 0 and "key.bias" not in k]
    groups = {
        "image conv (one vector)": [k for k in keys if k.startswith("image_encoder") and gb[k].dim() == 4],
        "image BN params": [k for k in keys if k.startswith("image_encoder") and gb[k].dim() == 1],
        "projections": [k for k in keys if k in ("image_projection", "text_projection")],
        "text tower": [k for k in keys if k.startswith("text_encoder")],
    }
    out = {}
    for name, ks in groups.items():
        va = torch.cat([ga[k].double().flatten() for k in ks])
        vb = torch.cat([gb[k].double().flatten() for k in ks])
        out[name] = rel(va, vb)
    return out


@pytest.fixture(scope="module")
def runs256():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sd = module_init_state()
    batch = synth_batch(256, 512, 40, 11)
    probe = batch["x-ray"][:32]
    return hip_bf16(sd, batch, probe), cpu_oracle(sd, batch, probe)


def test_bf16_loss_features_embeddings_bs256(runs256):
    hip, ora = runs256
    d = abs(hip["loss"] - ora["loss"])
    rf, ri, rt = rel(hip["feats"], ora["feats"]), rel(hip["ie"], ora["ie"]), rel(hip["te"], ora["te"])
    print(f"bs=256 512px T=40: loss bf16 {hip['loss']:.6f} fp32 {ora['loss']:.6f} |d|={d:.2e}; "
          f"probe features rel {rf:.2e}; img emb rel {ri:.2e}; txt emb rel {rt:.2e}")
    assert d <= 5e-2
    assert rf <= 2e-2 and ri <= 2e-2 and rt <= 2e-2


def tensor_errors(ga, gb):
    """rel-L2 per parameter tensor (same exclusions as group_errors)."""
    return {k: rel(ga[k], gb[k]) for k in gb if k in ga and gb[k].norm() > 0 and "key.bias" not in k}


def test_bf16_gradients_bs256(runs256):
    hip, ora = runs256
    errs = group_errors(hip["grads"], ora["grads"])
    print("bs=256 bf16 vs fp32 oracle gradient groups:", {k: round(v, 4) for k, v in errs.items()})
    for k, v in errs.items():
        assert v <= 0.30, (k, v)
    # per tensor: a single wrong layer (e.g. a downsample weight gradient) is not
    # diluted by its group.  Conv / projection / text weights carry many terms and
    # stay close to their group's error; BN parameters are sums of cancelling
    # terms (relative bf16 error up to ~0.5 on a handful of them)
    te = tensor_errors(hip["grads"], ora["grads"])
    worst = sorted(te.items(), key=lambda kv: -kv[1])[:8]
    print("bs=256 worst tensors:", [(k, round(v, 3)) for k, v in worst])
    for k, v in te.items():
        is_bn = ora["grads"][k].dim() == 1 and k.startswith("image_encoder")
        assert v <= (0.8 if is_bn else 0.4), (k, v)
    assert statistics.median(te.values()) <= 0.1


def test_bf16_gradients_vs_torch_autocast():
    """Per gradient group: err(HIP bf16, fp32) <= 1.5 * err(torch CPU bf16 autocast, fp32) + 0.01."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sd = module_init_state()
    batch = synth_batch(16, 256, 40, 12)
    hip = hip_bf16(sd, batch)
    ref = cpu_oracle(sd, batch)
    ac = cpu_oracle(sd, batch, autocast=True)
    e_hip, e_ac = group_errors(hip["grads"], ref["grads"]), group_errors(ac["grads"], ref["grads"])
    print("bs=16 256px vs fp32: hip bf16", {k: round(v, 4) for k, v in e_hip.items()},
          "| torch autocast bf16", {k: round(v, 4) for k, v in e_ac.items()})
    for k in e_hip:
        assert e_hip[k] <= 1.5 * e_ac[k] + 0.01, (k, e_hip[k], e_ac[k])
    assert abs(hip["loss"] - ref["loss"]) <= 5e-2
    assert statistics.mean(e_hip.values()) <= statistics.mean(e_ac.values()) * 1.5 + 0.01
    # embeddings: the text tower keeps its residual stream in bf16 like autocast's
    # matmul outputs; its deviation must stay within autocast's own
    r_img = (rel(hip["ie"], ref["ie"]), rel(ac["ie"], ref["ie"]))
    r_txt = (rel(hip["te"], ref["te"]), rel(ac["te"], ref["te"]))
    print(f"bs=16 embeddings rel-L2 (hip, autocast): image {r_img[0]:.2e} {r_img[1]:.2e}; "
          f"text {r_txt[0]:.2e} {r_txt[1]:.2e}")
    assert r_img[0] <= 1.5 * r_img[1] + 5e-3, r_img
    assert r_txt[0] <= 1.5 * r_txt[1] + 5e-3, r_txt
    # per tensor against torch's own per-tensor autocast error
    t_hip, t_ac = tensor_errors(hip["grads"], ref["grads"]), tensor_errors(ac["grads"], ref["grads"])
    excess = sorted(((t_hip[k] - (1.5 * t_ac[k] + 0.02), k, t_hip[k], t_ac[k]) for k in t_hip), reverse=True)
    print("bs=16 per-tensor worst (excess, name, hip, autocast):", [(round(a, 3), k, round(b, 3), round(c, 3))
                                                                   for a, k, b, c in excess[:5]])
    assert excess[0][0] <= 0, excess[:3]


def live_residual_state(seed):
    """Module init with every image-tower BatchNorm made live: gamma ~ U(0.3, 1.0),
    beta ~ U(-0.1, 0.1) (seeded).  timm's zero_init_last sets each block's
    bn2.weight = 0, which zeroes the gradients of conv1 / bn1 / conv2 of all 16
    blocks (32 of the 36 conv weights) -- a bf16 test from that init checks
    none of the residual-branch backward."""
    sd = module_init_state()
    g = torch.Generator().manual_seed(seed)
    for k, v in sd.items():
        if not k.startswith("image_encoder") or v.dim() != 1 or "running" in k:
            continue
        if k.endswith(".weight"):
            sd[k] = torch.empty_like(v).uniform_(0.3, 1.0, generator=g)
        elif k.endswith(".bias"):
            sd[k] = torch.empty_like(v).uniform_(-0.1, 0.1, generator=g)
    return sd


@pytest.mark.parametrize("bs,side,u8", [(16, 256, False), (8, 512, True)], ids=["bs16-256px-fp32in", "bs8-512px-u8"])
def test_bf16_live_residual_per_tensor_vs_autocast(bs, side, u8):
    """bf16 step with live residual branches, every parameter tensor gated on its
    own: err(HIP bf16, fp32) <= 1.5 x err(torch CPU bf16 autocast, fp32) + 0.02.

    No tensor is left out: the fp32 gradient of every conv weight (36) and every
    BN parameter must be non-zero.  The only exclusion is the text attention key
    bias, whose gradient is zero in exact arithmetic (softmax is invariant to a
    per-query constant); for it the HIP gradient (bf16 rounding noise of a sum
    of cancelling terms) must stay below 2 % of the query bias gradient.

    bs16-256px-fp32in: the reference's fp32 3-channel batch (K = 256 stem), the
    generic 64-wide layer-1 tiles.  bs8-512px-u8: the bench's path -- the uint8
    1-channel upload, the fused single-channel stem (forward pooling + Gram-form
    backward), the W = 128 layer-1 rows kernel with bn1 + ReLU in conv2's ring
    (vlp_conv_fwd_act) and its data-gradient epilogues."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sd = live_residual_state(100 + side)
    batch = synth_batch(bs, side, 40, 21 + side, with_u8=u8)
    hip_batch = dict(batch)
    if u8:
        hip_batch.pop("x-ray")
    hip = hip_bf16(sd, hip_batch)
    ref = cpu_oracle(sd, batch)
    ac = cpu_oracle(sd, batch, autocast=True)
    convs = [k for k in ref["grads"] if k.startswith("image_encoder") and ref["grads"][k].dim() == 4]
    bns = [k for k in ref["grads"] if k.startswith("image_encoder") and ref["grads"][k].dim() == 1]
    assert len(convs) == 36 and len(bns) == 72, (len(convs), len(bns))
    zero = [k for k in convs + bns if ref["grads"][k].norm() == 0]
    assert not zero, zero
    missing = [k for k in ref["grads"] if k not in hip["grads"]]
    assert not missing, missing
    kb = [k for k in ref["grads"] if "key.bias" in k]
    for k in kb:
        qb = k.replace("key.bias", "query.bias")
        assert hip["grads"][k].norm() <= 2e-2 * hip["grads"][qb].norm() + 1e-9, (k, hip["grads"][k].norm())
    names = [k for k in ref["grads"] if k not in kb]
    # a zeroed or non-finite HIP gradient fails here, whatever its rel-L2 gate says
    bad = [k for k in names if hip["grads"][k].norm() == 0 or not torch.isfinite(hip["grads"][k]).all()]
    assert not bad, bad
    # direction: a sign-flipped or zeroed gradient has cos ~ -c / 0.
    # In this small-batch regime a bf16 rounding next to a ReLU's zero flips its mask and
    # the gradient error grows like the square root of the flip rate, so torch's own
    # autocast reaches only cos ~0.7 on some BN parameters and two bf16 implementations
    # scatter around each other by ~0.05-0.1 in cosine: the gate is 0.8 x autocast's
    # cosine - 0.02 (the per-kernel sharp check is tests/test_gpu_blocks.py)
    c_hip = {k: cosine(hip["grads"][k], ref["grads"][k]) for k in names}
    c_ac = {k: cosine(ac["grads"][k], ref["grads"][k]) for k in names}
    worst_c = sorted(((c_hip[k] - (0.8 * c_ac[k] - 0.02), k, c_hip[k], c_ac[k]) for k in names))
    print("  cosine worst (margin, name, hip, autocast):",
          [(round(a, 4), k, round(b, 4), round(c, 4)) for a, k, b, c in worst_c[:4]])
    assert worst_c[0][0] >= 0, worst_c[:3]
    t_hip = {k: rel(hip["grads"][k], ref["grads"][k]) for k in names}
    t_ac = {k: rel(ac["grads"][k], ref["grads"][k]) for k in names}
    excess = sorted(((t_hip[k] - (1.5 * t_ac[k] + 0.02), k, t_hip[k], t_ac[k]) for k in names), reverse=True)
    print(f"\nbs={bs} {side}px live residual: loss hip {hip['loss']:.6f} fp32 {ref['loss']:.6f} "
          f"autocast {ac['loss']:.6f}")
    for sel, label in ((convs, "conv"), (bns, "BN")):
        worst = max(sel, key=lambda k: t_hip[k])
        print(f"  {label}: worst hip {worst} {t_hip[worst]:.4f} (autocast {t_ac[worst]:.4f}); "
              f"median hip {statistics.median(t_hip[k] for k in sel):.4f} "
              f"autocast {statistics.median(t_ac[k] for k in sel):.4f}")
    print("  per-tensor worst (excess, name, hip, autocast):",
          [(round(a, 4), k, round(b, 4), round(c, 4)) for a, k, b, c in excess[:6]])
    assert abs(hip["loss"] - ref["loss"]) <= 5e-2
    assert excess[0][0] <= 0, excess[:3]

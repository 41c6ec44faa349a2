"""NesT image tower (vlp_amd/nest.py) and the NesT + TinyBERT contrastive step
against the plain-torch restatement of timm nest_small (oracle/nest.py; timm
itself is absent, so NesT parity is UNPINNED against timm -- these tests pin the
HIP path to the restatement, whose layout/keys match timm's).

Shapes: img 64 (patch grid 16: 16 blocks of 4x4 tokens, 4 blocks at level 1, 1
at level 2), img 96 (blocks of 6x6 = 36 tokens: partial attention tiles) and
img 128 (8x8 = 64-token blocks: one full tile).  Weights: the tower's own timm
initialisation, copied into the oracle.  DropPath (timm default rate 0.5) is
exercised in train mode by replaying the tower's per-sample masks in the oracle.

Tolerances: fp32 features rel-L2 <= 1e-4 against the fp64 oracle and every
parameter gradient rel-L2 <= 1e-3 (GELU / softmax / LayerNorm are smooth; only
a max-pool tie could move a gradient discontinuously); bf16 features <= 5e-2 (24 layers of bf16 activations; measured 3.2e-2),
gradients <= 0.3 per tensor (torch bf16 autocast: up to 13 % on the level-0
parameters) and median <= 2e-2.
"""
import functools

import pytest
import torch

from tests.golden.synth import synth_batch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def make_pair(img, dtype, seed=0):
    import oracle.nest as on
    from vlp_amd.nest import NestTower
    torch.manual_seed(seed)
    t = NestTower("nest_small", img_size=img, compute_dtype=dtype, device="cuda")
    o = on.nest_small(img_size=img).double()
    o.load_state_dict({k: v.detach().double().cpu() for k, v in t.state_dict().items()})
    return t, o


def replay_masks(tower, oracle_model):
    """Feed the tower's last DropPath masks to the oracle's layers."""
    masks = tower.last_drop_masks
    for i, lvl in enumerate(oracle_model.levels):
        for j, layer in enumerate(lvl.transformer_encoder):
            m = masks[i][j] if masks is not None else None
            layer.masks = None if m is None else (m[0].double(), m[1].double())


@pytest.mark.parametrize("img", [64, 96, 128])
def test_tower_fp32_vs_oracle(img):
    t, o = make_pair(img, "fp32", seed=img)
    g = torch.Generator().manual_seed(img)
    x = torch.randn(2, 3, img, img, generator=g)
    # eval features (the linear-probe embedding)
    t.eval(); o.eval()
    with torch.no_grad():
        f = t(x.cuda())
        fo = o(x.double())
    assert rel(f, fo) < 1e-4, rel(f, fo)
    # train step with DropPath: features and every parameter gradient
    t.train(); o.train()
    w = torch.randn(2, 384, generator=g)
    f = t(x.cuda())
    (f * w.cuda()).sum().backward()
    replay_masks(t, o)
    fo = o(x.double())
    (fo * w.double()).sum().backward()
    assert rel(f.detach(), fo.detach()) < 1e-4
    og = dict(o.named_parameters())
    worst = max((rel(p.grad, og[k].grad), k) for k, p in t.named_parameters() if og[k].grad is not None
                and og[k].grad.norm() > 0)
    assert worst[0] < 1e-3, worst


def test_tower_bf16_vs_oracle():
    t, o = make_pair(128, "bf16", seed=5)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 128, 128, generator=g)
    t.train(); o.train()
    w = torch.randn(2, 384, generator=g)
    f = t(x.cuda())
    (f * w.cuda()).sum().backward()
    replay_masks(t, o)
    fo = o(x.double())
    (fo * w.double()).sum().backward()
    ef = rel(f.detach(), fo.detach())
    assert ef < 5e-2, ef
    og = dict(o.named_parameters())
    errs = sorted((rel(p.grad, og[k].grad), k) for k, p in t.named_parameters() if og[k].grad is not None
                  and og[k].grad.norm() > 0)
    # the level-0 parameters sit behind 24 residual layers: torch's own bf16
    # autocast of the oracle (same weights, input and DropPath rates) is 11-13 %
    # off fp64 on exactly these (pos_embed 13.3 %, patch_embed 12.3 %, fc1/norm2
    # of level 0 11-12 %); this path keeps the residual stream in bf16 too
    assert errs[-1][0] < 0.3, errs[-3:]
    assert errs[len(errs) // 2][0] < 2e-2, errs[len(errs) // 2]


def test_tower_bf16_512px_features():
    """BASELINE configs[3]'s resolution (512^2: 16 level-0 blocks of 32 x 32 tokens),
    B = 1: the bf16 tower's eval features against the fp32 oracle (rel-L2 <= 5e-2,
    the bf16 tower gate above)."""
    import oracle.nest as on
    from vlp_amd.nest import NestTower
    torch.manual_seed(9)
    t = NestTower("nest_small", img_size=512, compute_dtype="bf16", device="cuda")
    o = on.nest_small(img_size=512)
    o.load_state_dict({k: v.detach().float().cpu() for k, v in t.state_dict().items()})
    t.eval(); o.eval()
    x = torch.randn(1, 3, 512, 512, generator=torch.Generator().manual_seed(9))
    with torch.no_grad():
        f = t(x.cuda()).float()
        fo = o(x)
    ef = rel(f, fo)
    print(f"NesT bf16 512px B=1 eval features rel-L2 {ef:.3e}")
    assert ef < 5e-2, ef


def test_uint8_input_matches_float():
    t, _ = make_pair(64, "fp32", seed=2)
    t.eval()
    g = torch.Generator().manual_seed(2)
    xu = torch.randint(0, 256, (2, 1, 64, 64), generator=g, dtype=torch.uint8)
    xf = ((xu.float() - 127.5) / 73.9).expand(2, 3, 64, 64).contiguous()
    with torch.no_grad():
        a = t(xu.cuda())
        b = t(xf.cuda())
    assert rel(a, b) < 1e-6


def test_clip_step_nest_tinybert_vs_oracle():
    """The VisionLanguageModule step with image_model="nest_small" (BASELINE
    configs[3]: NesT-Small + TinyBERT) in fp32 against the oracle's step: loss
    and every gradient (eval-mode BN-free tower: DropPath off via drop_path_rate=0,
    text dropout off)."""
    from oracle.clip import OracleVLP, compute_loss
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    torch.manual_seed(0)
    m = VisionLanguageModule("nest_small", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False,
                             False, 384, 312, 128, compute_dtype="fp32", text_dropout=0.0, image_size=64,
                             drop_path_rate=0.0)
    m.train()
    o = OracleVLP(128, text_dropout=0.0, image_model="nest_small", img_size=64).double()
    sd = {k: v.detach().double().cpu() for k, v in m.state_dict().items()}
    missing = o.load_state_dict(sd, strict=False)
    assert not missing.unexpected_keys, missing.unexpected_keys
    o.train()
    for lvl in o.image_encoder.model.levels:
        for layer in lvl.transformer_encoder:
            layer.drop_path = 0.0
    b = synth_batch(6, 64, 12, 11)
    loss, li, lt, ie, te = m.training_step_outputs(b)
    loss.backward()
    bo = {"x-ray": b["x-ray"].double(), "caption_tokenized": b["caption_tokenized"]}
    logits, _, _ = o(bo)
    lo, _, _ = compute_loss(logits)
    lo.backward()
    assert abs(loss.item() - lo.item()) < 1e-5, (loss.item(), lo.item())
    og = dict(o.named_parameters())
    # attention.self.key.bias: adding a constant to every key of a query leaves the
    # softmax unchanged, so its true gradient is 0 and both sides hold rounding noise
    worst = max((rel(p.grad, og[k].grad), k) for k, p in m.named_parameters()
                if p.grad is not None and og[k].grad is not None and og[k].grad.norm() > 0
                and not k.endswith("attention.self.key.bias"))
    assert worst[0] < 2e-3, worst


def test_clip_step_nest_tinybert_bf16_256px():
    """BASELINE configs[3]'s workload in its compute dtype: the bf16 NesT-Small +
    TinyBERT contrastive step (text tower on its own stream, as the bench runs
    it) at 256^2 (level-0 blocks of 1024 tokens: the 512^2 block size) against
    the fp32 oracle on the same weights and batch.  DropPath off, text dropout
    off.  Loss |delta| <= 5e-2 and embeddings rel-L2 <= 5e-2.  At the module's
    init the contrastive logits are nearly uniform (loss ~ ln B), so every
    gradient is a difference of nearly equal embedding terms and bf16 rounding
    alone moves it by 10-40 %: each gradient tensor is therefore gated against
    torch's own CPU bf16 autocast run of the same oracle, err(HIP) <= 1.5 *
    err(autocast) + 0.02, as the ResNet34 step's test_bf16_gradients_vs_torch_autocast."""
    import statistics
    from oracle.clip import OracleVLP, compute_loss
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    torch.manual_seed(3)
    m = VisionLanguageModule("nest_small", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False,
                             False, 384, 312, 128, compute_dtype="bf16", text_dropout=0.0, image_size=256,
                             drop_path_rate=0.0)
    m.train()
    sd = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    b = synth_batch(4, 256, 40, 21, with_u8=True)
    bu = {"x-ray-u8": b["x-ray-u8"].cuda(), "label": b["label"], "caption": b["caption"],
          "caption_tokenized": {k: v.cuda() for k, v in b["caption_tokenized"].items()}}
    loss, li, lt, ie, te = m.training_step_outputs(bu)
    loss.backward()
    torch.cuda.synchronize()
    hip_g = {k: p.grad.float().cpu() for k, p in m.named_parameters() if p.grad is not None}

    def oracle(autocast):
        o = OracleVLP(128, text_dropout=0.0, image_model="nest_small", img_size=256)
        o.load_state_dict(sd, strict=False)
        o.train()
        for lvl in o.image_encoder.model.levels:
            for layer in lvl.transformer_encoder:
                layer.drop_path = 0.0
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            logits, oie, ote = o({"x-ray": b["x-ray"], "caption_tokenized": b["caption_tokenized"]})
        lo = compute_loss(logits.float())[0]
        lo.backward()
        return lo.item(), oie.detach().float(), ote.detach().float(), dict(o.named_parameters())

    lo, oie, ote, og = oracle(False)
    _, aie, ate, ag = oracle(True)
    d = abs(loss.item() - lo)
    ri, rt = rel(ie.float(), oie), rel(te.float(), ote)
    keys = [k for k in hip_g if og[k].grad is not None and og[k].grad.norm() > 0
            and not k.endswith("attention.self.key.bias")]
    e_hip = {k: rel(hip_g[k], og[k].grad) for k in keys}
    e_ac = {k: rel(ag[k].grad, og[k].grad) for k in keys}
    # The HIP tower stores NesT's residual stream (and its gradient) in bf16; torch
    # autocast adds every bf16 branch output into an fp32 residual (type promotion),
    # so the parameters behind the whole level-1/2 stack (level 0, patch / position
    # embedding: 20+ bf16 residual adds in each direction) carry up to ~0.2 rel-L2
    # more rounding than autocast's at this conditioning (near-uniform logits, the
    # gradient a small difference of nearly equal terms).  TinyBERT's residual
    # stream is bf16 as well.  Those keep the tower test's absolute 0.3 bound
    # (test_tower_bf16_vs_oracle); every other tensor is gated against autocast's
    # own per-tensor error, and the median over all tensors below.
    deep = ("image_encoder.model.levels.0.", "image_encoder.model.patch_embed", "text_encoder.")

    def tol(k):
        t = 1.5 * e_ac[k] + 0.02
        return max(t, 0.3) if k.startswith(deep) else t
    excess = sorted(((e_hip[k] - tol(k), k, e_hip[k], e_ac[k]) for k in keys), reverse=True)
    print(f"NesT bf16 256px: loss {loss.item():.5f} vs {lo:.5f}; emb rel {ri:.2e} / {rt:.2e} "
          f"(autocast {rel(aie, oie):.2e} / {rel(ate, ote):.2e}); grad median hip {statistics.median(e_hip.values()):.3e} "
          f"autocast {statistics.median(e_ac.values()):.3e}; worst excess "
          f"{[(round(a, 3), k, round(h, 3), round(c, 3)) for a, k, h, c in excess[:5]]}")
    assert d <= 5e-2 and ri <= 5e-2 and rt <= 5e-2
    assert excess[0][0] <= 0, excess[:3]
    assert statistics.median(e_hip.values()) <= 1.5 * statistics.median(e_ac.values()) + 0.01

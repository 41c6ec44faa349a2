"""Model-level parity: the HIP training step vs the CPU oracle and the
reference-generated golden vectors.

Tolerances (fp32 parity mode, stated per the north star):
  loss |delta| <= 1e-3 (observed ~1e-6), linear-probe features rel-L2 <= 1e-4,
  per-parameter gradient rel-L2 <= 2e-3, AdamW update rel <= 1e-2 (the update
  is ~lr*sign(g) on step 1, so it amplifies rounding of near-zero gradients).
bf16 throughput mode: loss |delta| <= 5e-2, features rel-L2 <= 5e-2 (measured
and reported, not the parity gate).
"""
import functools
import os

import pytest
import torch

from oracle import weights as W
from oracle.clip import OracleVLP, compute_loss
from tests.golden.synth import synth_batch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def make_model(dtype, seed=0):
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype=dtype, text_dropout=0.0)
    W.apply_recipe(m, seed)
    return m


def make_oracle(seed=0):
    o = OracleVLP(128, text_dropout=0.0)
    W.apply_recipe(o, seed)
    return o


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_probe_features_eval(dtype):
    B, H, T = 4, 64, 12
    batch = synth_batch(B, H, T, 0)
    gd = torch.load(os.path.join(GOLD, "step_B4_H64_T12.pt"), weights_only=True)
    m = make_model(dtype)
    m.eval()
    with torch.no_grad():
        f = m.image_encoder(batch["x-ray"].cuda())
    torch.cuda.synchronize()
    r = rel(f, gd["probe_features"])
    assert r < (1e-4 if dtype == "fp32" else 5e-2), r


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_train_step_vs_reference(dtype):
    B, H, T = 4, 64, 12
    gd = torch.load(os.path.join(GOLD, "step_B4_H64_T12.pt"), weights_only=True)
    batch = synth_batch(B, H, T, 0)
    m = make_model(dtype)
    m.train()
    opt = m.configure_optimizers()["optimizer"]
    loss = m.training_step(batch)
    dl = abs(loss.item() - gd["train_loss"].item())
    print(f"[{dtype}] loss {loss.item():.7f} ref {gd['train_loss'].item():.7f} |d|={dl:.2e}")
    assert dl < (1e-3 if dtype == "fp32" else 5e-2)
    loss.backward()
    names = gd["param_names"]
    params = dict(m.named_parameters())
    before = {k: params[k].detach().clone() for k in names}
    gn = [params[k].grad.norm().item() if params[k].grad is not None else -1.0 for k in names]
    if dtype == "fp32":
        # attention key biases have an exactly-zero gradient (softmax is shift invariant),
        # so both sides are rounding noise there: absolute floor 1e-6
        # early-layer gradients of this small-batch BN stack are ill-conditioned: the fp32
        # reference itself sits ~0.7% from fp64 there (tools/diag_grads.py), so norms are
        # compared at 2% here and element-wise against the fp64 envelope below
        worst = max((abs(a - b) / (abs(b) + 5e-4), k) for a, b, k in zip(gn, gd["grad_norm"].tolist(), names))
        print("worst grad-norm rel", worst)
        assert worst[0] < 2e-2, worst
    opt.step()
    torch.cuda.synchronize()
    dn = torch.tensor([(params[k].detach() - before[k]).norm().item() for k in names], dtype=torch.float64)
    if dtype == "fp32":
        r = rel(dn, gd["delta_norm"])
        assert r < 1e-2, r
    sd = m.state_dict()
    torch.testing.assert_close(sd["image_encoder.model.bn1.running_mean"].cpu(), gd["bn1_running_mean"],
                               rtol=1e-3 if dtype == "fp32" else 5e-2, atol=1e-5 if dtype == "fp32" else 1e-2)


def _oracle_step(batch, seed, dt):
    o = make_oracle(seed).to(dt)
    o.train()
    b = dict(batch)
    b["x-ray"] = batch["x-ray"].to(dt)
    lg, _, _ = o(b)
    lo = compute_loss(lg)[0]
    lo.backward()
    return o, lo


def grad_envelope_check(named_grads, o32, o64, strict):
    """Every parameter gradient vs the fp64 oracle, judged against the oracle's own
    fp32 error e_ref (err(HIP, fp64) <= 4 * e_ref, floor 2e-3 / 1e-6 absolute).

    strict=False (large shapes, recipe weights): a ReLU whose pre-activation lies
    within fp32 rounding of zero can take the other branch in HIP than in the
    oracle -- one such flip among ~1e5 activations moves the gradients of the
    layers below it by ~1e-3..1e-2 rel-L2, in either implementation (the fp32
    oracle itself sits 0.7 % from fp64 on these weights at 128 px, B = 8;
    tools/diag_blocks.py traces each such step to an exact upstream gradient and
    an op that matches torch to 2e-5 at that shape).  So per tensor the floor is
    2e-2, and the whole image-tower gradient (all 36 conv weights as one vector)
    must stay within max(2 x the fp32 oracle's own error, 5e-3) of fp64."""
    p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
    bad, hip_v, ref_v, o32_v = [], [], [], []
    floor = 2e-3 if strict else 2e-2
    for k, g in named_grads:
        g64 = p64[k].grad
        if g64 is None:
            assert g is None, k
            continue
        e_hip, e_ref = rel(g, g64), rel(p32[k].grad, g64)
        if e_hip > max(4 * e_ref, floor) and (g.double().cpu() - g64).norm().item() > 1e-6:
            bad.append((k, e_hip, e_ref))
        if k.startswith("image_encoder") and g64.dim() == 4:
            hip_v.append(g.double().cpu().flatten())
            ref_v.append(g64.double().flatten())
            o32_v.append(p32[k].grad.double().flatten())
    tower = rel(torch.cat(hip_v), torch.cat(ref_v))
    tower32 = rel(torch.cat(o32_v), torch.cat(ref_v))
    print(f"whole image-tower conv gradient rel-L2 vs fp64: hip {tower:.3e}, fp32 oracle {tower32:.3e}; "
          f"tensors over the envelope: {bad[:6]}")
    assert not bad, bad[:10]
    assert strict or tower <= max(2 * tower32, 5e-3), (tower, tower32)


@pytest.mark.parametrize("B,H,T", [(6, 96, 16), (2, 512, 40), (4, 224, 40)],
                         ids=["96px_T16", "bench_512px_T40", "ref_default_224px_T40"])
def test_grads_vs_oracle_fp32(B, H, T):
    """Parity mode vs the oracle: loss within 1e-5 of the fp64 oracle (north-star
    gate 1e-3), eval-mode probe features within rel-L2 1e-4, every gradient in
    the fp32 envelope (grad_envelope_check; strict at 96 px).  Shapes: 96x96 /
    T=16; the benchmark resolution and caption length (512x512, T=40: the W=128
    layer-1 rows kernel and the full-size stem run); the reference's own training
    resolution (224x224, PretrainDataModule.py:155; layer 1 is 56 wide there and
    takes the generic tile path)."""
    batch = synth_batch(B, H, T, 3)
    m = make_model("fp32", seed=1)
    o32p = make_oracle(1)
    m.eval()
    o32p.eval()
    with torch.no_grad():
        f = m.image_encoder(batch["x-ray"].cuda())
        fo = o32p.image_encoder(batch["x-ray"])
    torch.cuda.synchronize()
    assert rel(f, fo) < 1e-4, rel(f, fo)
    m.train()
    loss = m.training_step(batch)
    loss.backward()
    o32, l32 = _oracle_step(batch, 1, torch.float32)
    o64, l64 = _oracle_step(batch, 1, torch.float64)
    print(f"[{H}px T={T}] loss hip {loss.item():.8f} fp64 {l64.item():.8f} fp32 {l32.item():.8f}")
    assert abs(loss.item() - l64.item()) < 1e-5
    grad_envelope_check([(k, p.grad) for k, p in m.named_parameters()], o32, o64, strict=H <= 96)
    o = o32
    # running statistics after one train-mode forward
    sd, osd = m.state_dict(), o.state_dict()
    for k in osd:
        if "running" in k:
            assert rel(sd[k], osd[k]) < 1e-4, k


def _oracle_obj(batch, seed, dt, w):
    o = make_oracle(seed).to(dt)
    o.train()
    b = dict(batch)
    b["x-ray"] = batch["x-ray"].to(dt)
    lg, _, _ = o(b)
    lo, li, lt = compute_loss(lg)
    (w[0] * lo + w[1] * li + w[2] * lt).backward()
    return o


@pytest.mark.parametrize("path", ["fused_step", "api"])
@pytest.mark.parametrize("w", [(0.0, 1.0, 0.0), (0.7, 0.0, 1.3)], ids=["image_loss_only", "mixed"])
def test_per_direction_loss_gradients_fp32(path, w):
    """image_loss and text_loss are autograd tensors in the
    reference (:550-552).  Backward of w0*loss + w1*image_loss + w2*text_loss
    through the fused training step (ClipStepFn reruns the head with per-direction
    weights) and through the API forward + _compute_loss (_SymCEFn), every
    gradient in the strict fp64 envelope of the oracle's same objective."""
    B, H, T = 6, 96, 16     # test_grads_vs_oracle_fp32's strict configuration
    batch = synth_batch(B, H, T, 3)
    m = make_model("fp32", seed=1)
    m.train()
    if path == "fused_step":
        loss, li, lt, _, _ = m.training_step_outputs(batch)
    else:
        logits, _, _ = m(batch)
        loss, li, lt = m._compute_loss(logits, deduplicate=False, masked=False)
    obj = w[1] * li + w[2] * lt
    if w[0]:
        obj = obj + w[0] * loss
    obj.backward()
    torch.cuda.synchronize()
    o32, o64 = _oracle_obj(batch, 1, torch.float32, w), _oracle_obj(batch, 1, torch.float64, w)
    grads = [(k, p.grad) for k, p in m.named_parameters()]
    assert all(g is not None and torch.isfinite(g).all() for k, g in grads if dict(o64.named_parameters())[k].grad
               is not None)
    grad_envelope_check(grads, o32, o64, strict=True)


def test_api_forward_and_compute_loss_fp32():
    B, H, T = 4, 64, 12
    gd = torch.load(os.path.join(GOLD, "step_B4_H64_T12.pt"), weights_only=True)
    batch = synth_batch(B, H, T, 0)
    m = make_model("fp32")
    m.train()
    logits, ie, te = m(batch)
    loss, li, lt = m._compute_loss(logits, deduplicate=False, masked=False)
    assert abs(loss.item() - gd["train_loss"].item()) < 1e-3
    torch.testing.assert_close(logits.detach().cpu(), gd["logits"].float(), rtol=1e-3, atol=1e-3)
    loss.backward()
    assert m.image_projection.grad is not None and m.logit_scale.grad is not None


@pytest.mark.parametrize("api", ["fused_step", "towers"])
def test_gradient_accumulation_semantics(api):
    """After the first backward p.grad aliases the flat grad arena.  With a
    torch optimizer (fused_optimizer=False) the trainer zeroes it in place
    (zero_grad(set_to_none=False)): the next backward must give the same
    gradient, not twice it; and a backward without zero_grad must accumulate
    (2x), as torch autograd does.  "towers" drives the encoders through their
    own autograd Functions (the API forward / FusionModule path)."""
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    B, H, T = 4, 64, 12
    batch = synth_batch(B, H, T, 0)
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0,
                             fused_optimizer=False)
    W.apply_recipe(m, 0)
    m.train()
    opt = m.configure_optimizers()["optimizer"]
    assert type(opt).__name__ == "AdamW"

    def backward():
        if api == "fused_step":
            m.training_step(batch).backward()
        else:
            logits, _, _ = m(batch)
            m._compute_loss(logits, deduplicate=False, masked=False)[0].backward()
        torch.cuda.synchronize()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    g1 = backward()
    opt.zero_grad(set_to_none=False)
    g2 = backward()
    g3 = backward()   # no zero_grad: accumulates
    assert g1.keys() == g2.keys() == g3.keys() and len(g1) > 100
    for k in g1:
        # attention key biases have an exactly-zero gradient (softmax shift invariance):
        # both runs are rounding noise there (~1e-10), hence the absolute floor
        atol = max(1e-6 * g1[k].abs().max().item(), 1e-8)
        torch.testing.assert_close(g2[k], g1[k], rtol=1e-5, atol=atol, msg=lambda s: f"{k}: {s}")
        torch.testing.assert_close(g3[k], 2 * g1[k], rtol=1e-5, atol=2 * atol, msg=lambda s: f"{k}: {s}")


def test_uint8_collation_path_matches_float():
    """The pinned-uint8 upload path (device-side normalise + replicate) equals the
    reference float batch path."""
    B, H, T = 4, 64, 12
    batch = synth_batch(B, H, T, 0, with_u8=True)
    m = make_model("fp32")
    m.eval()
    with torch.no_grad():
        l1 = m.training_step_outputs({k: v for k, v in batch.items() if k != "x-ray-u8"})[0].item()
        b2 = dict(batch)
        b2["x-ray-u8"] = batch["x-ray-u8"]
        l2 = m.training_step_outputs(b2)[0].item()
    assert abs(l1 - l2) < 1e-5


def test_fused_adamw_matches_torch_and_state_dict_roundtrip():
    """FusedAdamW (one vlp_adamw launch per arena span) follows torch.optim.AdamW
    over three steps on the reference's parameter groups; its state_dict holds
    torch's per-parameter {step, exp_avg, exp_avg_sq} and round-trips: a fresh
    optimizer resumed from it (or from a torch AdamW state dict) takes the same
    next step."""
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd.optim import FusedAdamW
    B, H, T = 4, 64, 12
    batch = synth_batch(B, H, T, 0)

    def model(fused):
        # the module's own init: its gradients are well conditioned, so the two runs stay
        # on one trajectory (the recipe weights' BN stack turns fp32 update rounding into
        # ~1 % gradient differences by step 2, see grad_envelope_check)
        torch.manual_seed(0)
        m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=1e-3),
                                 False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0,
                                 fused_optimizer=fused)
        m.train()
        return m, m.configure_optimizers()["optimizer"]

    def step(m, opt):
        opt.zero_grad()
        m.training_step(batch).backward()
        opt.step()
        torch.cuda.synchronize()

    def flat(m):
        # attention key biases have an exactly-zero true gradient (softmax shift invariance):
        # AdamW turns their rounding noise into +-lr steps, different in every run
        return torch.cat([p.detach().double().flatten().cpu() for k, p in m.named_parameters()
                          if "attention.self.key.bias" not in k])

    mf, of = model(True)
    mt, ot = model(False)
    assert isinstance(of, FusedAdamW) and type(ot) is torch.optim.AdamW
    p0 = flat(mf)
    for _ in range(3):
        step(mf, of)
        step(mt, ot)
    d_f, d_t = flat(mf) - p0, flat(mt) - p0
    # (the golden test pins step 1; by step 3 fp32 rounding of two equivalent update
    # formulas has moved near-zero gradients, whose AdamW steps are ~lr * sign)
    assert rel(d_f, d_t) < 3e-3, rel(d_f, d_t)
    sd = of.state_dict()
    st = next(iter(sd["state"].values()))
    assert set(st) == {"step", "exp_avg", "exp_avg_sq"} and float(st["step"]) == 3.0
    for src_sd, src_model in ((sd, mf), (ot.state_dict(), mt)):
        m2, o2 = model(True)
        m2.load_state_dict(src_model.state_dict())
        o2.load_state_dict(src_sd)
        ref = [p.detach().clone() for k, p in src_model.named_parameters() if "attention.self.key.bias" not in k]
        m_next, o_next = (mf, of) if src_model is mf else (mt, ot)
        step(m_next, o_next)
        step(m2, o2)
        assert rel(flat(m2) - torch.cat([r.double().flatten().cpu() for r in ref]),
                   flat(m_next) - torch.cat([r.double().flatten().cpu() for r in ref])) < 3e-3

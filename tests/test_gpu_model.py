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


def test_grads_vs_oracle_fp32():
    """Every parameter gradient, B=6, 96x96, T=16, judged against the fp32
    rounding envelope: err(HIP, oracle-fp64) <= 4 * err(oracle-fp32, oracle-fp64)
    (or <= 2e-3 / 1e-6 absolute, whichever is looser)."""
    B, H, T = 6, 96, 16
    batch = synth_batch(B, H, T, 3)
    m = make_model("fp32", seed=1)
    m.train()
    loss = m.training_step(batch)
    loss.backward()
    o32, l32 = _oracle_step(batch, 1, torch.float32)
    o64, l64 = _oracle_step(batch, 1, torch.float64)
    assert abs(loss.item() - l64.item()) < 1e-5
    p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
    bad = []
    for k, p in m.named_parameters():
        g64 = p64[k].grad
        if g64 is None:
            assert p.grad is None, k
            continue
        e_hip, e_ref = rel(p.grad, g64), rel(p32[k].grad, g64)
        if e_hip > max(4 * e_ref, 2e-3) and (p.grad.double().cpu() - g64).norm().item() > 1e-6:
            bad.append((k, e_hip, e_ref))
    assert not bad, bad[:10]
    o = o32
    # running statistics after one train-mode forward
    sd, osd = m.state_dict(), o.state_dict()
    for k in osd:
        if "running" in k:
            assert rel(sd[k], osd[k]) < 1e-4, k


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

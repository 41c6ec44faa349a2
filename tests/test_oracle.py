"""CPU: pin the oracle (oracle/) against golden vectors produced by the
reference's own code (tests/golden/make_golden.py) and the notebook
known-answer values."""
import os

import math

import pytest
import torch

from oracle import weights as W
from oracle.clip import (OracleVLP, clip_forward, compute_loss, precision_at_k, recall_at_k)
from tests.golden.synth import synth_batch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def head_inputs(B, seed):
    g = torch.Generator().manual_seed(1000 + seed)
    return torch.randn(B, 512, generator=g), torch.randn(B, 312, generator=g)


def test_known_answers_notebook():
    ka = load("known_answers.pt")
    loss, li, lt = compute_loss(ka["nb14_logits"])
    # value computed through the reference's _compute_loss
    assert abs(loss.item() - 0.8721213) < 1e-6
    torch.testing.assert_close(torch.stack([loss, li, lt]), ka["nb14"], rtol=0, atol=1e-7)
    loss, li, lt = compute_loss(ka["asym_logits"])
    assert abs(loss.item() - 0.3726629) < 1e-6
    torch.testing.assert_close(torch.stack([loss, li, lt]), ka["asym"], rtol=0, atol=1e-7)


def test_retrieval_metrics():
    ka = load("known_answers.pt")
    e = torch.tensor([[1, 1], [1, 1.1], [2, 1], [3, 1]], dtype=torch.float32)
    assert precision_at_k(e, torch.tensor([0, 0, 1, 1]), [1])[1] == ka["prec_k1"].item() == 1.0
    p = precision_at_k(ka["retr_img"], ka["retr_lab"], [3, 5, 10, 15])
    r = recall_at_k(ka["retr_img"], ka["retr_txt"], [3, 5, 10, 15])
    assert [p[k] for k in (3, 5, 10, 15)] == pytest.approx(ka["prec"].tolist(), abs=1e-7)
    assert [r[k] for k in (3, 5, 10, 15)] == pytest.approx(ka["recall"].tolist(), abs=1e-7)


@pytest.mark.parametrize("tag", ["head_B4_s0", "head_B8_s1", "head_B8_s2", "head_B256_s3"])
def test_head_against_reference(tag):
    gd = load(tag + ".pt")
    B, seed = int(gd["B"]), int(gd["seed"])
    f_img, f_txt = head_inputs(B, seed)
    f_img.requires_grad_()
    f_txt.requires_grad_()
    Pi = W.value_for("image_projection", (512, 128)).requires_grad_()
    Pt = W.value_for("text_projection", (312, 128)).requires_grad_()
    ls = gd["logit_scale"].clone().requires_grad_()
    logits, ie, te = clip_forward(f_img, f_txt, Pi, Pt, ls)
    loss, li, lt = compute_loss(logits)
    loss.backward()
    tol = dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(loss.detach(), gd["loss"], **tol)
    torch.testing.assert_close(li.detach(), gd["image_loss"], **tol)
    torch.testing.assert_close(lt.detach(), gd["text_loss"], **tol)
    torch.testing.assert_close(ls.grad, gd["d_logit_scale"], **tol)
    torch.testing.assert_close(Pi.grad[:16], gd["d_image_projection_rows16"], **tol)
    torch.testing.assert_close(Pt.grad[:16], gd["d_text_projection_rows16"], **tol)
    suffix = "" if B <= 8 else "_rows16"
    rows = slice(None) if B <= 8 else slice(0, 16)
    for k, v in (("logits", logits), ("img_emb", ie), ("txt_emb", te), ("d_f_img", f_img.grad),
                 ("d_f_txt", f_txt.grad)):
        torch.testing.assert_close(v.detach()[rows], gd[k + suffix], **tol)
    if "s2" in tag:  # clamped logit scale: exp(ln 150) > 100 => no gradient
        assert gd["d_logit_scale"].abs().item() == 0.0


@pytest.mark.parametrize("case", ["image_only", "mixed"])
def test_direction_gradients_against_reference(case):
    """head_dir_B8_s1.pt: gradients of image_loss alone and of 0.7 loss + 1.3
    text_loss, through the reference's forward + _compute_loss (:550-552)."""
    gd = load("head_dir_B8_s1.pt")
    B, seed = int(gd["B"]), int(gd["seed"])
    c = gd[case]
    f_img, f_txt = head_inputs(B, seed)
    f_img.requires_grad_()
    f_txt.requires_grad_()
    Pi = W.value_for("image_projection", (512, 128)).requires_grad_()
    Pt = W.value_for("text_projection", (312, 128)).requires_grad_()
    ls = torch.tensor([math.log(1 / 0.07)], dtype=torch.float64).requires_grad_()
    logits, ie, te = clip_forward(f_img, f_txt, Pi, Pt, ls)
    loss, li, lt = compute_loss(logits)
    wl, wi, wt = c["weights"].tolist()
    (wl * loss + wi * li + wt * lt).backward()
    tol = dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(f_img.grad, c["d_f_img"], **tol)
    torch.testing.assert_close(f_txt.grad, c["d_f_txt"], **tol)
    torch.testing.assert_close(ls.grad, c["d_logit_scale"], **tol)
    torch.testing.assert_close(Pi.grad[:16], c["d_image_projection_rows16"], **tol)
    torch.testing.assert_close(Pt.grad[:16], c["d_text_projection_rows16"], **tol)


def test_global_batch_definition():
    gd = load("gathered_N2048.pt")
    N = int(gd["world"]) * int(gd["B"])
    g = torch.Generator().manual_seed(int(gd["seed"]))
    ie = torch.nn.functional.normalize(torch.randn(N, int(gd["E"]), generator=g)).requires_grad_()
    te = torch.nn.functional.normalize(torch.randn(N, int(gd["E"]), generator=g)).requires_grad_()
    ls = torch.tensor([W.value_for("logit_scale", (1,)).item()], dtype=torch.float64,
                      requires_grad=True)
    logits = (ie @ te.T) * torch.clamp(ls.exp(), max=100)
    loss, li, lt = compute_loss(logits)
    loss.backward()
    torch.testing.assert_close(loss.detach(), gd["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ls.grad, gd["d_logit_scale"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ie.grad[:8], gd["d_img_rows_0_8"], rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(te.grad[:8], gd["d_txt_rows_0_8"], rtol=1e-4, atol=1e-8)


def test_full_step_against_reference():
    gd = load("step_B4_H64_T12.pt")
    B, H, T = int(gd["B"]), int(gd["H"]), int(gd["T"])
    torch.manual_seed(0)
    model = OracleVLP(embedding_dim=128, text_dropout=0.0)
    W.apply_recipe(model, int(gd["seed"]))
    batch = synth_batch(B, H, T, int(gd["data_seed"]))
    model.eval()
    with torch.no_grad():
        feats = model.image_encoder(batch["x-ray"])
        lg, _, _ = model(batch)
        eval_loss = compute_loss(lg)[0]
    torch.testing.assert_close(feats, gd["probe_features"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(eval_loss, gd["eval_loss"], rtol=1e-5, atol=1e-6)
    model.train()
    opt = torch.optim.AdamW(model.param_groups(), lr=5e-5)
    assert [g["name"] for g in opt.param_groups] == gd["group_names"]
    assert [sum(p.numel() for p in g["params"]) for g in opt.param_groups] == gd["group_sizes"].tolist()
    lg, ie, te = model(batch)
    loss = compute_loss(lg)[0]
    torch.testing.assert_close(loss.detach(), gd["train_loss"], rtol=1e-5, atol=1e-6)
    opt.zero_grad()
    loss.backward()
    names = gd["param_names"]
    params = dict(model.named_parameters())
    before = {k: params[k].detach().clone() for k in names}
    gn = torch.tensor([params[k].grad.norm().item() if params[k].grad is not None else -1.0
                       for k in names], dtype=torch.float64)
    torch.testing.assert_close(gn, gd["grad_norm"], rtol=2e-4, atol=1e-9)
    opt.step()
    dn = torch.tensor([(params[k].detach() - before[k]).norm().item() for k in names],
                      dtype=torch.float64)
    torch.testing.assert_close(dn, gd["delta_norm"], rtol=1e-3, atol=1e-9)
    sd = model.state_dict()
    torch.testing.assert_close(sd["image_encoder.model.bn1.running_mean"], gd["bn1_running_mean"])
    torch.testing.assert_close(sd["image_encoder.model.bn1.running_var"], gd["bn1_running_var"])


def test_prep_crop_pad_vs_reference_transforms():
    """oracle/prep.py's restatement of CropLargerDimension / PadToSquaredEdgeAverage
    against the reference's own transforms (tests/golden/make_prep_golden.py):
    exact, on the raw images and after the equalisation."""
    import numpy as np
    import oracle.prep as op
    gd = torch.load(os.path.join(GOLD, "prep_crop_pad.pt"), weights_only=True)
    for c in gd["cases"]:
        u8 = c["u8"].numpy()
        raw = torch.from_numpy(u8.astype(np.float32))[None]
        eq = torch.from_numpy(op.histogram_normalize(u8.astype(np.float32)))[None]
        assert torch.equal(op.pad_to_square_edge_average(op.crop_larger_dimension(raw))[0], c["raw"]), u8.shape
        assert torch.equal(op.pad_to_square_edge_average(op.crop_larger_dimension(eq))[0], c["eq"]), u8.shape

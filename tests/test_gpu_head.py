"""HIP contrastive head vs the reference's own outputs.

The fixtures tests/golden/head_B*.pt and gathered_N2048.pt were produced by the
reference's `forward` (src/models/pretrain/VisionLanguageModule.py:441-461) and
`_compute_loss` (:532-554) in the build container (tests/golden/make_golden.py).
Here the same inputs go through the product path of the training step:
`_project_normalize` (HIP GEMM + L2 norm) -> `vlp_clip_loss_fused` (one kernel:
global-batch InfoNCE forward + analytic backward) -> `_project_backward`.

Cases: B = 4, 8, 8 with exp(logit_scale) = 150 > 100 (the clamp: d logit_scale
must be exactly 0, :456-457), B = 256; and the 8-rank global batch (N = 2048)
run as 8 launches with offset = r*256, N = 2048 -- exactly what every rank of an
8-GPU job executes -- whose loss partials, gathered-embedding gradients
(reduce-scatter = sum over ranks) and d logit_scale (all-reduce) are summed
as the collectives would.

Tolerances (fp32 on both sides; the reference keeps logit_scale in fp64, which
promotes its logits and loss to fp64):
  loss, image/text loss   |delta| <= 1e-5
  embeddings, logits      rtol 1e-5, atol 1e-5
  feature / projection / embedding gradients   rtol 1e-4, atol 1e-6 * max|golden|
  d logit_scale           rel 1e-4 (exactly 0 when clamped)
"""
import math
import os

import pytest
import torch

from oracle import weights as W

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def load(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def head_inputs(B, seed):
    """The features make_golden.head_case drew (same generator, same order)."""
    g = torch.Generator().manual_seed(1000 + seed)
    return torch.randn(B, 512, generator=g), torch.randn(B, 312, generator=g)


def close(got, want, rtol, atol_rel, what):
    got, want = got.detach().double().cpu(), want.detach().double().cpu()
    atol = atol_rel * max(want.abs().max().item(), 1e-30)
    err = (got - want).abs().max().item()
    torch.testing.assert_close(got, want, rtol=rtol, atol=atol, msg=lambda m: f"{what}: {m}")
    return err


def make_head(logit_scale):
    from vlp_amd.clip_model import ClipHead
    dev = torch.device("cuda")
    head = ClipHead(512, 312, 128, "fp32", device=dev)
    with torch.no_grad():
        head.arena.view("image_projection").copy_(W.value_for("image_projection", (512, 128)))
        head.arena.view("text_projection").copy_(W.value_for("text_projection", (312, 128)))
        head.arena.view("logit_scale").copy_(logit_scale.float())
    return head


def run_head(head, f_img, f_txt, role_w=None):
    """The ClipStepFn head, world = 1: forward + fused loss + backward (role_w: the
    per-direction weights of the image_loss / text_loss gradients)."""
    from vlp_amd import ops
    from vlp_amd.clip_model import _project_backward, _project_normalize
    dev = torch.device("cuda")
    fi, ft = f_img.to(dev).contiguous(), f_txt.to(dev).contiguous()
    B, E = fi.shape[0], 128
    wT = head.wcopy()
    ie, inorm = _project_normalize(head, wT, fi, 512, 512, "image_projection", E)
    te, tnorm = _project_normalize(head, wT, ft, 312, 312, "text_projection", E)
    g_img = torch.zeros(B, E, device=dev)
    g_txt = torch.zeros(B, E, device=dev)
    small = torch.zeros(4, device=dev)
    ops.clip_loss_fused(B, B, E, 0, ie, te, head.arena.view("logit_scale"), g_img, g_txt, small[2:3],
                        small[0:2], role_w=role_w)
    out = torch.empty(3, device=dev)
    ops.clip_loss_finish(small[0:2], B, out)
    gs = torch.ones(1, device=dev)
    head.arena.grad.zero_()
    ops.scale(small[2:3], gs, head.arena.gview("logit_scale"))
    dfi = _project_backward(head, wT, fi, 512, 512, "image_projection", E, ie, inorm, g_img, gs)
    dft = _project_backward(head, wT, ft, 312, 312, "text_projection", E, te, tnorm, g_txt, gs)
    torch.cuda.synchronize()
    return {"loss": out[0], "image_loss": out[1], "text_loss": out[2], "img_emb": ie, "txt_emb": te,
            "d_f_img": dfi, "d_f_txt": dft, "d_logit_scale": head.arena.gview("logit_scale").clone(),
            "d_image_projection": head.arena.gview("image_projection").clone(),
            "d_text_projection": head.arena.gview("text_projection").clone()}


@pytest.mark.parametrize("tag", ["head_B4_s0", "head_B8_s1", "head_B8_s2", "head_B256_s3"])
def test_clip_loss_fused_vs_reference(tag):
    from src.models.pretrain.VisionLanguageModule import _LogitsFn
    gd = load(tag + ".pt")
    B, seed = int(gd["B"]), int(gd["seed"])
    f_img, f_txt = head_inputs(B, seed)
    head = make_head(gd["logit_scale"])
    r = run_head(head, f_img, f_txt)
    for k in ("loss", "image_loss", "text_loss"):
        d = abs(r[k].item() - gd[k].item())
        assert d <= 1e-5, (k, r[k].item(), gd[k].item())
    small = B <= 8
    rows = slice(None) if small else slice(0, 16)
    sfx = "" if small else "_rows16"
    close(r["img_emb"][rows], gd["img_emb" + sfx], 1e-5, 1e-5, "img_emb")
    close(r["txt_emb"][rows], gd["txt_emb" + sfx], 1e-5, 1e-5, "txt_emb")
    # logits through the module's API path (HIP GEMM + scale, :456-459)
    lg = _LogitsFn.apply(r["img_emb"], r["txt_emb"], head.arena.view("logit_scale"))
    close(lg[rows], gd["logits" + sfx], 1e-5, 1e-5, "logits")
    close(r["d_f_img"][rows], gd["d_f_img" + sfx], 1e-4, 1e-6, "d_f_img")
    close(r["d_f_txt"][rows], gd["d_f_txt" + sfx], 1e-4, 1e-6, "d_f_txt")
    close(r["d_image_projection"][:16], gd["d_image_projection_rows16"], 1e-4, 1e-6, "d_image_projection")
    close(r["d_text_projection"][:16], gd["d_text_projection_rows16"], 1e-4, 1e-6, "d_text_projection")
    for k in ("d_image_projection", "d_text_projection"):
        n, ng = r[k].norm().item(), gd[k + "_norm"].item()
        assert abs(n - ng) <= 1e-4 * ng, (k, n, ng)
    if not small:
        for k in ("d_f_img", "d_f_txt"):
            n, ng = r[k].norm().item(), gd[k + "_norm"].item()
            assert abs(n - ng) <= 1e-4 * ng, (k, n, ng)
    dls, gls = r["d_logit_scale"].item(), gd["d_logit_scale"].item()
    if gls == 0.0:   # clamped branch (exp(logit_scale) = 150 > 100): no gradient at all
        assert "s2" in tag and dls == 0.0, dls
    else:
        assert abs(dls - gls) <= 1e-4 * abs(gls), (dls, gls)


@pytest.mark.parametrize("case", ["image_only", "mixed"])
def test_clip_loss_fused_per_direction_vs_reference(case):
    """Gradients of image_loss alone and of 0.7 loss + 1.3 text_loss (the reference's
    image_loss / text_loss are autograd tensors, :550-552), made by the reference in
    tests/golden/make_golden.py (head_dir_B8_s1.pt): role weights w_r = w_loss + 2 w_r."""
    from vlp_amd.clip_model import role_weights
    gd = load("head_dir_B8_s1.pt")
    B, seed = int(gd["B"]), int(gd["seed"])
    c = gd[case]
    f_img, f_txt = head_inputs(B, seed)
    head = make_head(torch.tensor([math.log(1 / 0.07)]))   # the reference init (:111)
    dev = torch.device("cuda")
    wl, wi, wt = [torch.tensor(v, device=dev) for v in c["weights"].tolist()]
    r = run_head(head, f_img, f_txt, role_w=role_weights(wl, wi, wt, dev))
    close(r["d_f_img"], c["d_f_img"], 1e-4, 1e-6, "d_f_img")
    close(r["d_f_txt"], c["d_f_txt"], 1e-4, 1e-6, "d_f_txt")
    close(r["d_image_projection"][:16], c["d_image_projection_rows16"], 1e-4, 1e-6, "d_image_projection")
    close(r["d_text_projection"][:16], c["d_text_projection_rows16"], 1e-4, 1e-6, "d_text_projection")
    dls, gls = r["d_logit_scale"].item(), c["d_logit_scale"].item()
    assert abs(dls - gls) <= 1e-4 * abs(gls), (dls, gls)


def test_clip_loss_fused_global_batch_8_ranks():
    """The N = 2048 global batch of an 8-GPU job: each rank's launch covers its
    256 rows (image->text) and 256 columns (text->image) at offset r*256."""
    from vlp_amd import ops
    gd = load("gathered_N2048.pt")
    world, B, E, seed = int(gd["world"]), int(gd["B"]), int(gd["E"]), int(gd["seed"])
    N = world * B
    g = torch.Generator().manual_seed(seed)
    ie = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).cuda()
    te = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).cuda()
    ls = torch.tensor([W.value_for("logit_scale", (1,)).item()], device="cuda")
    parts = torch.zeros(2, dtype=torch.float64, device="cuda")
    dls = torch.zeros(1, dtype=torch.float64, device="cuda")
    g_img = torch.zeros(N, E, dtype=torch.float64, device="cuda")
    g_txt = torch.zeros(N, E, dtype=torch.float64, device="cuda")
    for r in range(world):
        gi = torch.zeros(N, E, device="cuda")
        gt = torch.zeros(N, E, device="cuda")
        small = torch.zeros(4, device="cuda")
        ops.clip_loss_fused(B, N, E, r * B, ie, te, ls, gi, gt, small[2:3], small[0:2])
        # the collectives of ClipStepFn: all-reduce of the loss partials and of the
        # head gradient (d logit_scale), reduce-scatter (= sum) of the gathered grads
        parts += small[0:2].double()
        dls += small[2:3].double()
        g_img += gi.double()
        g_txt += gt.double()
    torch.cuda.synchronize()
    loss = (parts[0] + parts[1]).item() / (2 * N)
    li, lt = parts[0].item() / N, parts[1].item() / N
    assert abs(loss - gd["loss"].item()) <= 1e-5, (loss, gd["loss"].item())
    assert abs(li - gd["image_loss"].item()) <= 1e-5, (li, gd["image_loss"].item())
    assert abs(lt - gd["text_loss"].item()) <= 1e-5, (lt, gd["text_loss"].item())
    gls = gd["d_logit_scale"].item()
    assert abs(dls.item() - gls) <= 1e-4 * abs(gls), (dls.item(), gls)
    close(g_img[:8], gd["d_img_rows_0_8"], 1e-4, 1e-6, "d_img rows 0-8")
    close(g_txt[:8], gd["d_txt_rows_0_8"], 1e-4, 1e-6, "d_txt rows 0-8")
    for k, t in (("d_img_norm", g_img), ("d_txt_norm", g_txt)):
        n, ng = t.norm().item(), gd[k].item()
        assert abs(n - ng) <= 1e-5 * ng, (k, n, ng)


def test_clip_loss_fused_deterministic_and_timed_N2048():
    """The split-key loss kernels use no atomics: two launches give bitwise-equal
    gradients.  Timed per rank at the 8-GPU global batch (B = 256, N = 2048,
    E = 128): the launch sits on the critical path between the embedding
    all-gather and the backward (the one-kernel version swept all N
    keys with 32 workgroups)."""
    from vlp_amd import ops
    B, N, E = 256, 2048, 128
    g = torch.Generator().manual_seed(5)
    ie = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).cuda()
    te = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).cuda()
    ls = torch.tensor([2.6592600], device="cuda")
    outs = []
    for _ in range(2):
        nan = float("nan")
        gi, gt = torch.full((N, E), nan, device="cuda"), torch.full((N, E), nan, device="cuda")
        small = torch.full((4,), nan, device="cuda")
        ops.clip_loss_fused(B, N, E, 3 * B, ie, te, ls, gi, gt, small[2:3], small[0:2])
        outs.append((gi, gt, small[:3].clone()))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        # every element written (no NaN of the fill survives), then bitwise equal
        assert not torch.isnan(a).any() and not torch.isnan(b).any()
        assert torch.equal(a, b)
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.clip_loss_fused(B, N, E, 3 * B, ie, te, ls, gi, gt, small[2:3], small[0:2])
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[5]
    print(f"clip_loss_fused per rank at N = 2048: {ms * 1e3:.1f} us")
    assert ms < 0.5, ms


@pytest.mark.parametrize("E", [32, 64, 200, 256])
def test_clip_loss_fused_embedding_dims(E):
    """every embedding width the kernels accept (E % 4 == 0, E <= 256;
    E = 256 takes the 16-chunk register tiles and ~130 KB of LDS in clip_dq; 200
    is not a multiple of 16) against a torch fp64 symmetric cross-entropy built
    here (reference forward :441-461, _compute_loss :532-554).  N = 101 split over
    three "ranks" of B = 37, 37, 27 (B not a multiple of 16, N not a multiple of
    64): their summed partials and gradients are the global-batch loss and its
    gradients, as the collectives of ClipStepFn form them."""
    from vlp_amd import ops
    F = torch.nn.functional
    N, Bs = 101, [37, 37, 27]
    g = torch.Generator().manual_seed(E)
    ie = F.normalize(torch.randn(N, E, generator=g, dtype=torch.float64))
    te = F.normalize(torch.randn(N, E, generator=g, dtype=torch.float64))
    ls = torch.tensor([2.3], dtype=torch.float64)
    x, y, l = ie.clone().requires_grad_(), te.clone().requires_grad_(), ls.clone().requires_grad_()
    s = torch.clamp(l.exp(), max=100.0)
    logits = s * x @ y.t()
    lab = torch.arange(N)
    li, lt = F.cross_entropy(logits, lab), F.cross_entropy(logits.t(), lab)
    ((li + lt) / 2).backward()
    parts = torch.zeros(2, dtype=torch.float64)
    dls = 0.0
    gi_all = torch.zeros(N, E, dtype=torch.float64)
    gt_all = torch.zeros(N, E, dtype=torch.float64)
    ied, ted = ie.float().cuda(), te.float().cuda()
    lsd = ls.float().cuda()
    off = 0
    for B in Bs:
        gi = torch.full((N, E), float("nan"), device="cuda")
        gt = torch.full((N, E), float("nan"), device="cuda")
        small = torch.zeros(4, device="cuda")
        ops.clip_loss_fused(B, N, E, off, ied, ted, lsd, gi, gt, small[2:3], small[0:2])
        torch.cuda.synchronize()
        assert not torch.isnan(gi).any() and not torch.isnan(gt).any()
        parts += small[0:2].double().cpu()
        dls += small[2].item()
        gi_all += gi.double().cpu()
        gt_all += gt.double().cpu()
        off += B
    assert abs(parts[0].item() / N - li.item()) <= 1e-5, (parts[0].item() / N, li.item())
    assert abs(parts[1].item() / N - lt.item()) <= 1e-5, (parts[1].item() / N, lt.item())
    close(gi_all, x.grad, 1e-4, 1e-6, f"d img emb E={E}")
    close(gt_all, y.grad, 1e-4, 1e-6, f"d txt emb E={E}")
    assert abs(dls - l.grad.item()) <= 1e-4 * abs(l.grad.item()), (dls, l.grad.item())

"""Cross-stream schedules must not change results.

The training step runs work on three HIP streams: the main stream (image
tower), the text-tower stream (TinyBERT forward/backward beside the image
tower, clip_model._USE_TEXT_STREAM) and, optionally, the image tower's
weight-gradient stream (resnet34._USE_WG_STREAM).  The split-K weight-gradient
workspaces (ops.wgrad_ws / ops._linw_ws) are per (device, stream); before that
fix the text stream's linear weight gradients and NesT's (main stream) shared
one buffer, as did the side-stream conv weight gradients and the main-stream
stem weight gradient.

Test A: bf16 ResNet34 + TinyBERT step, weight-gradient stream on vs off.  The
image tower's conv weight gradients come from deterministic split slabs, so
they must equal the stream-off result bit for bit, or within 4x the run-to-run
noise of two stream-off steps when that is not 0 (an fp64 BN-sum atomic landing
on a rounding boundary).
Test B: bf16 NesT + TinyBERT step at 64^2, text stream on vs off: every
gradient within max(1e-6, 4 x run-to-run noise of either schedule) rel-L2.
"""
import functools

import pytest
import torch

from tests.golden.synth import synth_batch

pytestmark = pytest.mark.gpu


def _grads(m, b):
    for p in m.parameters():
        p.grad = None
    loss, *_ = m.training_step_outputs(b)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_wgrad_stream_matches_serial_bf16():
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd import resnet34 as r34
    torch.manual_seed(0)
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False, False,
                             512, 312, 128, compute_dtype="bf16", text_dropout=0.0)
    m.train()
    # non-zero bn2 gammas so every block's gradient path is live
    with torch.no_grad():
        for k, p in m.named_parameters():
            if k.endswith("bn2.weight"):
                p.fill_(0.5)
    b = synth_batch(8, 128, 16, 3, with_u8=True)
    b = {"x-ray-u8": b["x-ray-u8"].cuda(), "label": b["label"], "caption": b["caption"],
         "caption_tokenized": {k: v.cuda() for k, v in b["caption_tokenized"].items()}}
    was = r34._USE_WG_STREAM
    try:
        r34._USE_WG_STREAM = False
        l0, g0 = _grads(m, b)
        l1, g1 = _grads(m, b)
        r34._USE_WG_STREAM = True
        l2, g2 = _grads(m, b)
        l3, g3 = _grads(m, b)
    finally:
        r34._USE_WG_STREAM = was
    conv = [k for k in g0 if k.startswith("image_encoder.") and (".conv" in k or "downsample.0" in k)]
    assert len(conv) == 36
    for k in conv:
        noise = (g0[k] - g1[k]).abs().max().item()
        for g in (g2, g3):
            d = (g[k] - g0[k]).abs().max().item()
            assert d <= 4 * noise, (k, d, noise)
    assert abs(l2 - l0) <= 4 * abs(l1 - l0) + 1e-7, (l0, l1, l2)


def test_text_stream_matches_serial_nest_bf16():
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd import clip_model as cm
    torch.manual_seed(1)
    m = VisionLanguageModule("nest_small", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False,
                             False, 384, 312, 128, compute_dtype="bf16", text_dropout=0.0, image_size=64,
                             drop_path_rate=0.0)
    m.train()
    b = synth_batch(8, 64, 24, 5, with_u8=True)
    b = {"x-ray-u8": b["x-ray-u8"].cuda(), "label": b["label"], "caption": b["caption"],
         "caption_tokenized": {k: v.cuda() for k, v in b["caption_tokenized"].items()}}
    was = cm._USE_TEXT_STREAM
    try:
        cm._USE_TEXT_STREAM = False
        l0, g0 = _grads(m, b)
        l1, g1 = _grads(m, b)
        cm._USE_TEXT_STREAM = True
        l2, g2 = _grads(m, b)
        l3, g3 = _grads(m, b)
    finally:
        cm._USE_TEXT_STREAM = was
    assert len(g0) > 300
    assert abs(l2 - l0) <= max(1e-6, 4 * abs(l1 - l0)), (l0, l1, l2)
    worst = []
    for k in g0:
        if g0[k].norm() == 0:
            continue
        # run-to-run noise of each schedule (fp32 atomics in the LayerNorm /
        # embedding backward reorder between runs)
        noise = max(_rel(g1[k], g0[k]), _rel(g3[k], g2[k]))
        tol = max(1e-6, 4 * noise)
        for g in (g2, g3):
            r = _rel(g[k], g0[k])
            worst.append((r - tol, k, r, tol))
    worst.sort()
    print("text stream on vs off, worst (excess, name, rel, tol):", worst[-3:])
    assert worst[-1][0] <= 0, worst[-3:]


@pytest.mark.parametrize("which", ["fwd", "bwd"])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_split_schedule_matches_unsplit(dtype, which):
    """Test C: the two-half, two-stream training forward (resnet34._SPLIT_FWD) or
    backward (_SPLIT_BWD: BN-backward passes and data gradients in halves, weight
    gradients on a third stream) against the one-stream schedule.  Both halves add into the same fp64 BN
    statistic replicas; what differs is the GEMM tiling the half-size launches
    pick (fp32 accumulation order).  fp32: loss within 1e-5 rel, every
    image-tower gradient within max(2e-3, 4 x unsplit run-to-run noise) rel-L2 (the
    fp32 envelope of tests/test_gpu_model.py: a ReLU pre-activation within
    rounding of 0 may flip) and the BN running statistics of one step from the
    same state within 1e-6 -- an ordering or half-indexing error would be O(1).
    bf16: the same step within bf16 tiling noise (loss 2e-3 rel, gradients 0.1)."""
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd import resnet34 as r34
    torch.manual_seed(2)
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False, False,
                             512, 312, 128, compute_dtype=dtype, text_dropout=0.0)
    m.train()
    with torch.no_grad():
        for k, p in m.named_parameters():
            if k.endswith("bn2.weight"):
                p.fill_(0.5)
    b = synth_batch(8, 128, 16, 4, with_u8=True)
    b = {"x-ray-u8": b["x-ray-u8"].cuda(), "label": b["label"], "caption": b["caption"],
         "caption_tokenized": {k: v.cuda() for k, v in b["caption_tokenized"].items()}}
    rm = {k: v for k, v in m.named_buffers() if k.endswith("running_mean") or k.endswith("running_var")}
    was = (r34._SPLIT_FWD, r34._SPLIT_BWD)
    flag = "_SPLIT_FWD" if which == "fwd" else "_SPLIT_BWD"
    try:
        r34._SPLIT_FWD = r34._SPLIT_BWD = False
        l0, g0 = _grads(m, b)
        r0 = {k: v.clone() for k, v in rm.items()}
        l1, g1 = _grads(m, b)
        r1 = {k: v.clone() for k, v in rm.items()}
        setattr(r34, flag, True)
        for k in rm:
            rm[k].copy_(r0[k])   # step 1 moved them: replay its update from the same state
        l2, g2 = _grads(m, b)
        r2 = {k: v.clone() for k, v in rm.items()}
    finally:
        r34._SPLIT_FWD, r34._SPLIT_BWD = was
    fp32 = dtype == "fp32"
    assert abs(l2 - l0) <= max((1e-5 if fp32 else 2e-3) * abs(l0), 4 * abs(l1 - l0)), (l0, l1, l2)
    img = [k for k in g0 if k.startswith("image_encoder.")]
    assert len(img) > 100
    worst = []
    for k in img:
        if g0[k].norm() == 0:
            continue
        tol = max(2e-3 if fp32 else 0.1, 4 * _rel(g1[k], g0[k]))
        r = _rel(g2[k], g0[k])
        worst.append((r - tol, k, r, tol))
    worst.sort()
    print(f"split {which} vs unsplit ({dtype}), worst (excess, name, rel, tol):", worst[-3:])
    assert worst[-1][0] <= 0, worst[-3:]
    if fp32:   # one momentum update from the same running state with the same batch statistics
        for k in rm:
            assert _rel(r2[k], r1[k]) <= 1e-6, (k, _rel(r2[k], r1[k]))

"""World-size-2 data-parallel step of the REAL HIP path vs the oracle's
per-rank-BN global-batch definition.

Two ranks (torch.distributed.run, gloo backend, both on the box's one GPU;
tests/_dp_worker.py) each run VisionLanguageModule.training_step + backward
in fp32 parity mode on their 4-row shard of an 8-row batch.  ClipStepFn then
does everything an 8-GPU job does: all-gather of the normalised embeddings,
the fused loss over the rank's rows/columns of the global 8 x 8 matrix
(offset = rank * 4), all-reduce of the loss partials, reduce-scatter of the
gathered-embedding gradients, and the bucketed all-reduce of the gradient
arenas (image tower per stage, text tower, head).

The definition it must equal: the oracle's image tower run per 4-row shard
(train-mode BN statistics per rank, as the reference's per-device BN), the
features concatenated, the text tower on all 8 captions, and the reference
_compute_loss on the 8 x 8 logits; gradients of that global loss.
Weights: the module's own initialisation (timm / HF init, what a training run
starts from), whose fp32 gradients are well conditioned (HIP fp32 vs the
oracle ~3e-6 single-GPU), so every non-zero gradient -- stem, downsample convs,
every BN parameter, projections, logit scale, the whole text tower -- is held to
the strict fp32 envelope.  (The recipe weights of the other parity tests make
this small-batch BN stack sensitive to single ReLU flips; see
test_gpu_model.grad_envelope_check.)
Tolerances: loss |delta| <= 1e-5 vs the fp64 oracle; every gradient inside
the strict fp32 envelope; both ranks hold bit-identical gradients after the
all-reduce.
"""
import os
import subprocess
import sys

import pytest
import torch

from oracle.clip import OracleVLP, compute_loss, clip_forward
from tests.conftest import ROOT
from tests.golden.synth import synth_batch

pytestmark = pytest.mark.gpu
B, H, T, SEED = 4, 64, 12, 5


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path_factory.mktemp("dp")
    # --standalone: torchrun binds its own free rendezvous port on 127.0.0.1 (a port
    # picked here and released before torchrun binds it can be taken in between:
    # EADDRINUSE seen once on a shared box)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", "--nproc-per-node", "2",
           os.path.join(ROOT, "tests", "_dp_worker.py"), str(out), str(B), str(H), str(T), str(SEED)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, env=env, timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [torch.load(out / f"r{k}.pt", weights_only=True) for k in range(2)]
    res[0]["init"] = torch.load(out / "init.pt", weights_only=True)
    return res


def _oracle(dt, sd):
    o = OracleVLP(128, text_dropout=0.0)
    o.load_state_dict(sd)
    o = o.to(dt)
    o.train()
    full = synth_batch(2 * B, H, T, SEED)
    x = full["x-ray"].to(dt)
    f_img = torch.cat([o.image_encoder(x[r * B:(r + 1) * B]) for r in range(2)])   # per-rank BN
    f_txt = o.text_encoder(**full["caption_tokenized"])
    logits, _, _ = clip_forward(f_img, f_txt, o.image_projection, o.text_projection, o.logit_scale)
    loss, li, lt = compute_loss(logits)
    loss.backward()
    return o, loss.item(), li.item(), lt.item()


def test_dp2_loss_is_global_batch_loss(ranks):
    _, l64, li64, lt64 = _oracle(torch.float64, ranks[0]["init"])
    for r in ranks:
        assert abs(r["loss"] - l64) <= 1e-5, (r["loss"], l64)
        assert abs(r["image_loss"] - li64) <= 1e-5
        assert abs(r["text_loss"] - lt64) <= 1e-5


def test_dp2_gradients_are_global_gradients(ranks):
    g0, g1 = ranks[0]["grads"], ranks[1]["grads"]
    assert g0.keys() == g1.keys()
    for k in g0:
        assert torch.equal(g0[k], g1[k]), f"ranks disagree after the all-reduce: {k}"
    from tests.test_gpu_model import grad_envelope_check
    o32, _, _, _ = _oracle(torch.float32, ranks[0]["init"])
    o64, _, _, _ = _oracle(torch.float64, ranks[0]["init"])
    assert len(g0) > 100
    p64 = dict(o64.named_parameters())
    named = [(k, g0.get(k)) for k in p64 if p64[k].grad is not None or k in g0]
    grad_envelope_check(named, o32, o64, strict=True)

"""Diagnostic: the NesT + TinyBERT bf16 step with the text stream off / on (as
tests/test_gpu_streams.py B); prints per-parameter differences against the
run-to-run noise of each schedule (top 12) and per-tower summaries."""
import functools
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
from tests.golden.synth import synth_batch  # noqa: E402


def grads(m, b):
    for p in m.parameters():
        p.grad = None
    loss, *_ = m.training_step_outputs(b)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
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
    runs = []
    for on in (False, False, True, True, False, True):
        cm._USE_TEXT_STREAM = on
        runs.append((on, *grads(m, b)))
    print("losses:", [(on, round(l, 7)) for on, l, _ in runs])
    g0, g1, g2, g3 = (r[2] for r in runs[:4])
    rows = []
    for k in g0:
        noise = max(rel(g1[k], g0[k]), rel(g3[k], g2[k]))
        d = max(rel(g2[k], g0[k]), rel(g3[k], g0[k]))
        rows.append((d - 4 * noise, k, d, noise, g0[k].norm().item()))
    rows.sort()
    for r in rows[-12:]:
        print("excess %.3e %s diff %.3e noise %.3e norm %.3e" % (r[0], r[1], r[2], r[3], r[4]))
    for k in ("text_projection", "image_projection", "logit_scale", "text_encoder.model.embeddings.LayerNorm.weight",
              "text_encoder.model.encoder.layer.3.output.dense.weight",
              "image_encoder.model.levels.2.transformer_encoder.7.norm1.weight"):
        print(k, "norms off/off/on/on:", ["%.4e" % r[2][k].norm().item() for r in runs[:4]])
    for tower in ("image_encoder", "text_encoder"):
        ks = [k for k in g0 if k.startswith(tower)]
        print(tower, "bitwise off==off:", sum(torch.equal(g0[k], g1[k]) for k in ks), "on==on:",
              sum(torch.equal(g2[k], g3[k]) for k in ks), "on==off:", sum(torch.equal(g2[k], g0[k]) for k in ks),
              "of", len(ks))


if __name__ == "__main__":
    main()

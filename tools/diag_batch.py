"""bf16 vs fp32 gradient error as a function of batch size / resolution, and the
fp32 HIP path vs the fp32 CPU oracle.  Same recipe weights (seed 2), same batch.
  python tools/diag_batch.py H:B[:oracle] ...     e.g. 512:2 256:64 512:256 128:32:oracle
Per config: loss of each path, rel-L2 of the projection gradients and the
median / max over the 36 conv weight gradients, per stage."""
import functools
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from oracle import weights as W  # noqa: E402
from oracle.clip import OracleVLP, compute_loss  # noqa: E402
from tests.golden.synth import synth_batch  # noqa: E402
from src.models.pretrain.VisionLanguageModule import VisionLanguageModule  # noqa: E402


BN2 = float(os.environ.get("DIAG_BN2", "1.0"))   # scale of every block's bn2 gamma


def scale_bn2(model):
    with torch.no_grad():
        for k, p in model.named_parameters():
            if k.endswith("bn2.weight"):
                p.mul_(BN2)


INIT = os.environ.get("DIAG_INIT", "recipe")   # recipe | timm (the module's own init, as the bench)
_SD = {}


def init_weights(model):
    if INIT == "recipe":
        W.apply_recipe(model, 2)
        scale_bn2(model)
        return
    if "sd" not in _SD:
        torch.manual_seed(0)
        _SD["sd"] = {k: v.detach().cpu().clone() for k, v in VisionLanguageModule(
            "resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5), False, False, 512, 312, 128,
            compute_dtype="fp32", text_dropout=0.0).state_dict().items()}
    model.load_state_dict(_SD["sd"])


def hip_grads(dt, batch):
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype=dt, text_dropout=0.0)
    init_weights(m)
    m.train()
    loss = m.training_step(batch)
    loss.backward()
    torch.cuda.synchronize()
    g = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters() if p.grad is not None}
    l = loss.item()
    del m
    torch.cuda.empty_cache()
    return l, g


def oracle_grads(batch):
    o = OracleVLP(128, text_dropout=0.0)
    init_weights(o)
    o.train()
    lg, _, _ = o(batch)
    loss = compute_loss(lg)[0]
    loss.backward()
    return loss.item(), {k: p.grad.detach().double() for k, p in o.named_parameters() if p.grad is not None}


def report(tag, la, ga, lb, gb):
    def rel(k):
        return ((ga[k] - gb[k]).norm() / (gb[k].norm() + 1e-30)).item()
    gb = {k: v for k, v in gb.items() if v.norm() > 0}
    allk = [k for k in gb if k.startswith("image_encoder") and gb[k].dim() == 4]
    va = torch.cat([ga[k].flatten() for k in allk])
    vb = torch.cat([gb[k].flatten() for k in allk])
    bnk = [k for k in gb if k.startswith("image_encoder") and gb[k].dim() == 1]
    print(f"== {tag}: image BN params: median rel {statistics.median(rel(k) for k in bnk):.3e} "
          f"max {max(rel(k) for k in bnk):.3e}; nonzero conv grads {len(allk)}")
    print(f"== {tag} [init {INIT} bn2 x{BN2}]: whole-tower conv-gradient rel-L2 {((va - vb).norm() / vb.norm()).item():.3e}")
    print(f"== {tag}: loss {la:.6f} vs {lb:.6f} |d| {abs(la - lb):.2e}", flush=True)
    for k in ("image_projection", "text_projection", "logit_scale"):
        print(f"   {k:18s} rel {rel(k):.3e}  |g| {gb[k].norm().item():.3e}")
    for st in ("conv1.", "layer1", "layer2", "layer3", "layer4"):
        ks = [k for k in gb if k.startswith("image_encoder.model." + st) and gb[k].dim() == 4]
        if not ks:
            continue
        rs = [rel(k) for k in ks]
        worst = max(zip(rs, ks))
        print(f"   {st:7s} conv median {statistics.median(rs):.3e} max {worst[0]:.3e} ({worst[1][20:]})"
              f"  |g| {gb[worst[1]].norm().item():.3e}")
    tk = [k for k in gb if k.startswith("text_encoder") and "key.bias" not in k and gb[k].norm() > 1e-12]
    rs = sorted(((rel(k), k) for k in tk), reverse=True)
    print(f"   text    median {statistics.median(r for r, _ in rs):.3e} max {rs[0][0]:.3e} ({rs[0][1][19:]})")


for spec in sys.argv[1:]:
    parts = spec.split(":")
    H, B = int(parts[0]), int(parts[1])
    batch = synth_batch(B, H, 40, 11)
    l32, g32 = hip_grads("fp32", batch)
    if len(parts) > 2 and parts[2] == "oracle":
        lo, go = oracle_grads(batch)
        report(f"{H}px B={B} HIP fp32 vs CPU oracle fp32", l32, g32, lo, go)
    l16, g16 = hip_grads("bf16", batch)
    report(f"{H}px B={B} HIP bf16 vs HIP fp32", l16, g16, l32, g32)

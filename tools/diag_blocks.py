"""Where does the fp32 HIP image-tower gradient leave the oracle?  Per block:
the gradient w.r.t. the block output (HIP, stashed by ResNet34Tower._dbg) vs the
fp64 oracle's; per parameter: HIP-fp32 and oracle-fp32 errors vs fp64.
  python tools/diag_blocks.py H B T [seed] [batch_seed]"""
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402
from oracle import weights as W  # noqa: E402
from oracle.clip import OracleVLP, compute_loss  # noqa: E402
from oracle.resnet34 import BasicBlock  # noqa: E402
from tests.golden.synth import synth_batch  # noqa: E402
from src.models.pretrain.VisionLanguageModule import VisionLanguageModule  # noqa: E402

H, B, T = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 1
bseed = int(sys.argv[5]) if len(sys.argv) > 5 else 3
batch = synth_batch(B, H, T, bseed)

m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                         False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0)
W.apply_recipe(m, seed)
m.train()
tower = m.image_encoder.model
tower._dbg = {}
loss = m.training_step(batch)
loss.backward()
torch.cuda.synchronize()
hip_g = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters() if p.grad is not None}


def oracle(dt):
    o = OracleVLP(128, text_dropout=0.0)
    W.apply_recipe(o, seed)
    o = o.to(dt)
    o.train()
    outs = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            outs[name] = out
        return hook
    for li in range(1, 5):
        for bi, blk in enumerate(getattr(o.image_encoder.model, f"layer{li}")):
            pre = f"layer{li}.{bi}"
            blk.register_forward_hook(keep(pre))
            blk.conv2.register_forward_hook(keep(pre + "/dy2"))   # grad of conv2 output = dy2
            blk.conv1.register_forward_hook(keep(pre + "/dy1"))
            blk.bn1.register_forward_hook(keep(pre + "/bn1out"))
    b = dict(batch)
    b["x-ray"] = batch["x-ray"].to(dt)
    lg, _, _ = o(b)
    lo = compute_loss(lg)[0]
    lo.backward()
    return o, lo.item(), outs


o64, l64, outs64 = oracle(torch.float64)
o32, l32, outs32 = oracle(torch.float32)
print(f"loss hip {loss.item():.9f} fp64 {l64:.9f} fp32 {l32:.9f}")
print("block output gradients (rel-L2 vs fp64): hip | oracle-fp32")
for name, (d, masked) in sorted(tower._dbg.items(), key=lambda kv: kv[0]):
    oname = name.replace("/g1", "/bn1out")
    out = outs64[oname]
    g64 = out.grad.permute(0, 2, 3, 1)
    if masked or name.endswith("/g1"):   # g1 = d relu(bn1) output * (bn1 output > 0)
        g64 = g64 * (out.detach().permute(0, 2, 3, 1) > 0)
    g32 = outs32[oname].grad.permute(0, 2, 3, 1).double()
    if masked or name.endswith("/g1"):
        g32 = g32 * (outs32[oname].detach().permute(0, 2, 3, 1) > 0)
    r = ((d.double().cpu() - g64).norm() / g64.norm()).item()
    r32 = ((g32 - g64).norm() / g64.norm()).item()
    print(f"  {name:10s} masked={int(masked)}  {r:.3e} | {r32:.3e}")
p64, p32 = dict(o64.named_parameters()), dict(o32.named_parameters())
print("parameters with hip error > max(4*oracle-fp32 error, 2e-3):")
for k, g in hip_g.items():
    if not k.startswith("image_encoder"):
        continue
    ref = p64[k].grad.double()
    e = ((g - ref).norm() / (ref.norm() + 1e-300)).item()
    e32 = ((p32[k].grad.double() - ref).norm() / (ref.norm() + 1e-300)).item()
    if e > max(4 * e32, 2e-3):
        print(f"  {k[20:]:32s} hip {e:.3e} fp32-oracle {e32:.3e} |g| {ref.norm().item():.3e}")

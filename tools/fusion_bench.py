"""Late-fusion finetune step (BASELINE configs[4]: ResNet34 Imaging+Clinical, bs=512,
512x512, bf16) on the HIP ResNet34 tower: images/s for forward + backward + AdamW.

    python tools/fusion_bench.py [--batch 512] [--steps 10] [--warmup 3] [--out F]

One process per GPU; under torch.distributed.run each rank takes its own bs and the
gradients are SUM-all-reduced (one RCCL call over the tower's flat gradient arena,
one over the head's ~6.7k gradients) and scaled by 1/world, as DDP's mean.  The
batch is resident in HBM (uint8 1-channel upload, normalised on the device).
"""
import argparse
import functools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GFLOP_PER_IMAGE = 113.60   # ResNet34 fwd+bwd (no input grad) at 512^2, SURVEY §8(d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--coral-lambda", type=float, default=0.5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    from src.models.baseline.FusionModule import FusionModule
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    m = FusionModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-4, fused=True),
                     label_weights=(0.6, 1.8), coral_lambda=a.coral_lambda, compute_dtype="bf16")
    opt = m.configure_optimizers()["optimizer"]
    B, H = a.batch, a.image_size
    g = torch.Generator().manual_seed(1 + rank)
    oh = torch.nn.functional.one_hot
    batch = {"x-ray-u8": torch.randint(0, 256, (B, 1, H, H), generator=g, dtype=torch.uint8).to(dev),
             "tumor": torch.randint(0, 2, (B,), generator=g).to(dev),
             "dataset": ["INTERNAL" if i % 3 else "BTXRD" for i in range(B)],
             "anatomy_site_encoded": oh(torch.randint(0, 9, (B,), generator=g), 9).float().to(dev),
             "age_encoded": oh(torch.randint(0, 4, (B,), generator=g), 4).float().to(dev),
             "sex_encoded": oh(torch.randint(0, 2, (B,), generator=g), 2).float().to(dev)}
    head = [p for n, p in m.named_parameters() if not n.startswith("image_network.") or ".fc." in n]

    def step():
        opt.zero_grad(set_to_none=False)
        loss = m.training_step(batch)
        loss.backward()
        if world > 1:
            dist.all_reduce(m.image_network.arena.grad)
            flat = torch.cat([p.grad.reshape(-1) for p in head])
            dist.all_reduce(flat)
            m.image_network.arena.grad.mul_(1.0 / world)
            off = 0
            for p in head:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad)).mul_(1.0 / world)
                off += n
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    ips = world * B * a.steps / el
    res = {"metric": "images/s (fwd+bwd+AdamW), ResNet34 Imaging+Clinical late-fusion finetune",
           "value": round(ips, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(el / a.steps * 1e3, 3), "dtype": "bf16", "data": "synthetic",
           "config": {"workload": "BASELINE configs[4] FusionModule resnet34", "per_gpu_batch": B,
                      "image_size": H, "coral_lambda": a.coral_lambda},
           "model_flops_frac": round(ips * GFLOP_PER_IMAGE * 1e9 / (world * 2.5e15), 4),
           "loss": round(loss.item(), 5)}
    if rank == 0:
        line = json.dumps(res)
        print(line)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Worker of tests/test_gpu_dp.py (not collected by pytest): one rank of a
world-size-2 data-parallel training step of the real HIP path.

Launched by torch.distributed.run with the gloo backend, both ranks on the
one GPU of the test box (vlp_amd.dist stages device tensors through host
memory under gloo).  Each rank takes its B-row shard of a 2B-row synthetic
batch, runs VisionLanguageModule.training_step + backward (ClipStepFn:
embedding all-gather, fused global-batch loss, reduce-scatter, bucketed
gradient all-reduce) in fp32 parity mode, and writes its loss terms and every
parameter gradient to <outdir>/r<rank>.pt.
"""
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    outdir, B, H, T, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from oracle import weights as W
    from tests.golden.synth import synth_batch
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule

    torch.cuda.set_device(0)
    torch.manual_seed(0)   # the module's own init, identical on both ranks
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0)
    if os.environ.get("DP_INIT", "module") == "recipe":
        W.apply_recipe(m, 1)
    if rank == 0:
        torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, os.path.join(outdir, "init.pt"))
    m.train()
    full = synth_batch(world * B, H, T, seed)
    sl = slice(rank * B, (rank + 1) * B)
    batch = {"x-ray": full["x-ray"][sl], "label": full["label"][sl],
             "caption_tokenized": {k: v[sl] for k, v in full["caption_tokenized"].items()}}
    loss, li, lt, ie, te = m.training_step_outputs(batch)
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters() if p.grad is not None}
    torch.save({"loss": loss.item(), "image_loss": li.item(), "text_loss": lt.item(),
                "img_emb": ie.detach().cpu(), "txt_emb": te.detach().cpu(), "grads": grads},
               os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

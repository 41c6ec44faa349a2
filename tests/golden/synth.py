"""Synthetic radiograph/caption batches, shared by the golden
generator, the tests, the bench and the CPU baseline.

Images: per-sample uint8 1-channel HxW ~ U{0..255} (seeded), normalised with
(x - 127.5) / 73.9 and replicated to 3 channels (PretrainDataModule.py:165-171).
Captions: input_ids [B, T] = CLS(101), L ~ U{8..20} content tokens
~ U{1000..29999}, SEP(102), PAD(0); attention_mask 1 on the first L+2
positions; token_type_ids 0.  Labels ~ Bernoulli(0.5).
"""
import torch

IMG_MEAN, IMG_STD = 127.5, 73.9


def synth_images_u8(B, H, seed=0, W=None):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, 1, H, W or H), generator=g, dtype=torch.uint8)


def normalize_u8(x_u8):
    x = (x_u8.float() - IMG_MEAN) / IMG_STD
    return x.repeat(1, 3, 1, 1).contiguous()


def synth_captions(B, T, seed=1):
    g = torch.Generator().manual_seed(seed)
    ids = torch.zeros(B, T, dtype=torch.long)
    mask = torch.zeros(B, T, dtype=torch.long)
    for b in range(B):
        L = int(torch.randint(8, 21, (1,), generator=g))
        L = min(L, T - 2)
        ids[b, 0] = 101
        ids[b, 1:1 + L] = torch.randint(1000, 30000, (L,), generator=g)
        ids[b, 1 + L] = 102
        mask[b, :L + 2] = 1
    return {"input_ids": ids, "token_type_ids": torch.zeros_like(ids), "attention_mask": mask}


def synth_batch(B, H, T, seed=0, with_u8=False):
    x_u8 = synth_images_u8(B, H, seed)
    g = torch.Generator().manual_seed(seed + 17)
    batch = {
        "x-ray": normalize_u8(x_u8),
        "caption_tokenized": synth_captions(B, T, seed + 1),
        "label": torch.randint(0, 2, (B,), generator=g),
        "caption": [f"synthetic caption {i}" for i in range(B)],
    }
    if with_u8:
        batch["x-ray-u8"] = x_u8
    return batch

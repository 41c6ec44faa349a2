"""Drop-in for the reference's src/data/PretrainDataModule.py on MI355X:
batch collation into pinned host memory and an asynchronous host-to-device
prefetcher, the collation row of SURVEY §8(a).

Reference behaviour kept:
  * constructor kwargs batch_size / num_workers / num_channels / tokenizer /
    try_with_only_n_samples / disable_augmentations (PretrainDataModule.py:89-98);
    num_channels not in {1, 3} raises ValueError (:111-114);
  * the batch schema handed to VisionLanguageModule (:141-149, :318-326 with
    torch default_collate): "x-ray" [B,3,H,W] fp32 normalised and replicated to
    3 channels (:165-171), "caption_tokenized" {input_ids, token_type_ids,
    attention_mask} [B,T] int64 padded to at most 40 tokens (:210-215), "label"
    [B], and the string lists "caption", "dataset", "anatomy_site", "image_path";
  * get_cv_splits() yields (datamodule, label_weights) (:270), train_dataloader()
    with pin_memory=True, val_dataloader() -> [lera_val, mura_val] (:318-350).

MI355X-first changes:
  * upload="u8" (default) collates the 1-channel uint8 radiograph as
    "x-ray-u8" [B,1,H,W] (67 MB per bs=256 512^2 batch instead of 805 MB of
    fp32); the module normalises and replicates it on the device
    (vlp_stem_prep_u8).  upload="fp32" reproduces the reference tensor.
  * DevicePrefetcher copies batch i+1 to HBM on a side HIP stream while step i
    runs and hands it over with a stream-ordered event wait, so the PCIe copy
    is off the step's critical path.
  * image_size (default 224, the reference's) and the synthetic dataset.

  * the training augmentations run on the device (device_augment ->
    vlp_amd.augment, csrc/prep_ops.hip), called by the trainer on each training
    batch after the upload; vlp_amd.augment.preprocess is the device form of the
    pre-normalisation chain (histogram equalisation, crop, pad, area resize) for
    decoded radiographs of any size.

The MURA/LERA readers and caption sampler need datasets that are not in this
image; with synthetic=False the module raises NotImplementedError.  Synthetic samples
follow SURVEY §8(d): uint8 pixels ~ U{0..255} (histogram-equalised), captions
CLS + U{8..20} tokens in [1000, 30000) + SEP, zero padding.
"""
from __future__ import annotations

import logging
from typing import Iterable, Iterator, List, Optional

import torch
from torch.utils.data import DataLoader, Dataset

logger = logging.getLogger("project")

IMG_MEAN, IMG_STD = 127.5, 73.9   # (x - mean) / std after HistogramNormalized -> [0, 255]
CLS_ID, SEP_ID, PAD_ID = 101, 102, 0
MAX_TOKENS = 40                    # tokenizer max_length (:213)
_SITES = ("ELBOW", "FINGER", "FOREARM", "HAND", "HUMERUS", "SHOULDER", "WRIST", "FOOT", "KNEE", "HIP")


def normalize_u8(x_u8: torch.Tensor, num_channels: int = 3, mean: float = IMG_MEAN,
                 std: float = IMG_STD) -> torch.Tensor:
    """uint8 [B,1,H,W] -> fp32 [B,C,H,W]: (x - mean) / std, channel replicated (:165-171)."""
    x = (x_u8.float() - mean) / std
    return x.repeat(1, num_channels, 1, 1).contiguous() if num_channels != 1 else x.contiguous()


class SyntheticRadiographCaptions(Dataset):
    """Seeded per-sample radiograph/caption dicts in the reference's sample layout."""

    def __init__(self, n: int, image_size: int, seq_len: int = MAX_TOKENS, seed: int = 0,
                 dataset_name: str = "MURA"):
        if seq_len < 3 or seq_len > MAX_TOKENS:
            raise ValueError(f"seq_len must be in [3, {MAX_TOKENS}], got {seq_len}")
        self.n, self.H, self.T, self.seed, self.name = n, image_size, seq_len, seed, dataset_name

    def __len__(self):
        return self.n

    def __getitem__(self, i: int) -> dict:
        if not 0 <= i < self.n:
            raise IndexError(i)
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        img = torch.randint(0, 256, (1, self.H, self.H), generator=g, dtype=torch.uint8)
        L = min(int(torch.randint(8, 21, (1,), generator=g)), self.T - 2)
        ids = torch.full((self.T,), PAD_ID, dtype=torch.long)
        ids[0] = CLS_ID
        ids[1:1 + L] = torch.randint(1000, 30000, (L,), generator=g)
        ids[1 + L] = SEP_ID
        mask = torch.zeros(self.T, dtype=torch.long)
        mask[:L + 2] = 1
        label = int(torch.randint(0, 2, (1,), generator=g))
        site = _SITES[int(torch.randint(0, len(_SITES), (1,), generator=g))]
        return {
            "x-ray-u8": img,
            "caption_tokenized": {"input_ids": ids, "token_type_ids": torch.zeros_like(ids),
                                  "attention_mask": mask},
            "label": label,
            "caption": f"synthetic {site.lower()} radiograph {i}",
            "dataset": self.name,
            "anatomy_site": site,
            "image_path": f"synthetic://{self.name}/{i}.png",
        }


class PairCollator:
    """Per-sample dicts -> the batch dict VisionLanguageModule consumes (default_collate layout).

    mean / std: the intensity normalisation (the reference's NormalizeIntensityd with
    the fold's dataset statistics, PretrainDataModule.py:283-288).  The fp32 upload
    applies it on the host; the u8 upload carries it as "x-ray-u8-norm" (two host
    floats) and the module applies it on the device (vlp_stem_prep_u8)."""

    def __init__(self, upload: str = "u8", num_channels: int = 3, mean: float = IMG_MEAN, std: float = IMG_STD):
        if upload not in ("u8", "fp32"):
            raise ValueError(f"upload must be 'u8' or 'fp32', got {upload!r}")
        self.upload, self.num_channels = upload, num_channels
        self.mean, self.std = float(mean), float(std)

    def __call__(self, samples: List[dict]) -> dict:
        if not samples:
            raise ValueError("empty batch")
        x_u8 = torch.stack([s["x-ray-u8"] for s in samples])
        batch = {
            "caption_tokenized": {k: torch.stack([s["caption_tokenized"][k] for s in samples])
                                  for k in ("input_ids", "token_type_ids", "attention_mask")},
            "label": torch.tensor([s["label"] for s in samples], dtype=torch.long),
        }
        for k in ("caption", "dataset", "anatomy_site", "image_path"):
            batch[k] = [s[k] for s in samples]
        if self.upload == "u8":
            if self.num_channels != 3:
                raise ValueError("the u8 upload feeds the 3-channel ImageNet-layout stem")
            batch["x-ray-u8"] = x_u8
            batch["x-ray-u8-norm"] = (self.mean, self.std)
        else:
            batch["x-ray"] = normalize_u8(x_u8, self.num_channels, self.mean, self.std)
        return batch


def _to_device(obj, device, stream):
    if torch.is_tensor(obj):
        return obj.to(device, non_blocking=True)
    if isinstance(obj, dict):
        return {k: _to_device(v, device, stream) for k, v in obj.items()}
    return obj


def _record(obj, stream):
    if torch.is_tensor(obj):
        obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record(v, stream)


_COPY_STREAMS = {}


def _copy_stream(device):
    """One upload stream per device shared by every prefetcher (a new stream per
    epoch / iterator would keep adding streams onto the process's few hardware
    queues)."""
    s = _COPY_STREAMS.get(device)
    if s is None:
        s = _COPY_STREAMS[device] = torch.cuda.Stream(device=device)
    return s


class DevicePrefetcher:
    """Iterates host batches (pinned) and yields device-resident batches.

    Batch i+1 is copied on a dedicated copy stream while the caller's stream
    runs step i; each yielded batch is made visible to the consumer stream by
    an event wait (no host synchronisation) and its tensors are recorded on the
    consumer stream so the caching allocator does not recycle them early.
    On a CPU device the batches pass through unchanged.
    """

    def __init__(self, loader: Iterable[dict], device, depth: int = 1):
        self.loader, self.device, self.depth = loader, torch.device(device), max(1, depth)

    def __iter__(self) -> Iterator[dict]:
        if self.device.type != "cuda":
            yield from self.loader
            return
        copy_stream = _copy_stream(self.device)
        pending = []
        it = iter(self.loader)

        def launch():
            try:
                host = next(it)
            except StopIteration:
                return False
            with torch.cuda.stream(copy_stream):
                dev = _to_device(host, self.device, copy_stream)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            pending.append((dev, ev))
            return True

        for _ in range(self.depth):
            if not launch():
                break
        while pending:
            dev, ev = pending.pop(0)
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            _record(dev, cur)
            launch()
            yield dev


class PretrainDataModule:
    def __init__(
        self,
        captions_path: Optional[str] = None,
        batch_size: int = 32,
        num_workers: int = 2,
        num_channels: int = 3,
        tokenizer: str = "distilbert",
        try_with_only_n_samples: Optional[int] = None,
        disable_augmentations: bool = False,
        image_size: int = 224,
        synthetic: bool = True,
        n_samples: int = 1024,
        n_val_samples: int = 64,
        seq_len: int = MAX_TOKENS,
        upload: str = "u8",
        seed: int = 0,
        drop_last: bool = True,
    ):
        if not (num_channels == 1 or num_channels == 3):
            raise ValueError(f"PretrainDataModule: num_channels must be 1 or 3, but got {num_channels}")
        if tokenizer not in ("distilbert", "tinybert"):
            raise ValueError(f"PretrainDataModule: unsupported tokenizer {tokenizer!r}")
        if not synthetic:
            raise NotImplementedError(
                "PretrainDataModule (MI355X build): the MURA/LERA readers and MONAI augmentations are "
                "not part of this build; use synthetic=True")
        if upload == "u8" and num_channels != 3:
            upload = "fp32"
        self.batch_size, self.num_workers, self.num_channels = batch_size, num_workers, num_channels
        self.tokenizer = tokenizer
        self.try_with_only_n_samples = try_with_only_n_samples
        self.disable_augmentations = disable_augmentations
        self.image_size, self.seq_len, self.upload, self.seed = image_size, seq_len, upload, seed
        self.drop_last = drop_last
        n = n_samples if try_with_only_n_samples is None else min(n_samples, try_with_only_n_samples)
        nv = n_val_samples if try_with_only_n_samples is None else min(n_val_samples, try_with_only_n_samples)
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        self.train_dataset = SyntheticRadiographCaptions(n, image_size, seq_len, seed + 7919 * rank, "MURA")
        self.val_datasets = [SyntheticRadiographCaptions(nv, image_size, seq_len, seed + 1_000 + rank, "LERA"),
                             SyntheticRadiographCaptions(nv, image_size, seq_len, seed + 2_000 + rank, "MURA")]
        # per-fold intensity statistics of the training images (the reference computes and
        # caches them per fold, :217-267, for NormalizeIntensityd)
        self.image_mean, self.image_std = self._intensity_stats(self.train_dataset)
        self.collate = PairCollator(upload, num_channels, self.image_mean, self.image_std)
        self._augmenter = None
        if disable_augmentations:
            logger.warning("PretrainDataModule: No augmentations are applied.")

    def device_augment(self, batch: dict) -> dict:
        """The reference's training augmentations (RandAffined, RandRotated, RandFlipd,
        RandZoomd, RandGaussianNoised; PretrainDataModule.py:186-198) on a device batch
        in one pass (vlp_amd.augment.Augmenter -> vlp_aug_warp): the uint8 upload is
        normalised on load and comes back as the fp32 "x-ray" tensor.  Identity when
        augmentations are disabled or the batch is on the CPU."""
        if self.disable_augmentations:
            return batch
        x = batch.get("x-ray-u8", batch.get("x-ray"))
        if x is None or x.device.type != "cuda":
            return batch
        if self._augmenter is None:
            from vlp_amd.augment import Augmenter
            rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
            self._augmenter = Augmenter(seed=self.seed * 1_000_003 + 17 * rank + 1)
        out = dict(batch)
        if "x-ray-u8" in batch:
            out["x-ray"] = self._augmenter(x, channels=self.num_channels, mean=self.image_mean, std=self.image_std)
            del out["x-ray-u8"]
            out.pop("x-ray-u8-norm", None)
        else:
            out["x-ray"] = self._augmenter(x, channels=self.num_channels)
        return out

    @staticmethod
    def _intensity_stats(ds, n: int = 64):
        """Mean / std of the (histogram-equalised) uint8 pixels over up to n training
        images; the synthetic U{0..255} pixels give ~127.5 / 73.9."""
        k = min(n, len(ds))
        if k == 0:
            return IMG_MEAN, IMG_STD
        x = torch.stack([ds[i]["x-ray-u8"] for i in range(k)]).double()
        return float(x.mean()), float(x.std())

    def get_cv_splits(self):
        """(:270) one split; label weights (1, 1) as the pretraining experiments use."""
        yield self, (1.0, 1.0)

    def _loader(self, ds, shuffle):
        return DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle, num_workers=self.num_workers,
                          collate_fn=self.collate, pin_memory=torch.cuda.is_available(),
                          drop_last=self.drop_last and shuffle, persistent_workers=False)

    def train_dataloader(self) -> DataLoader:
        return self._loader(self.train_dataset, True)

    def val_dataloader(self) -> List[DataLoader]:
        return [self._loader(ds, False) for ds in self.val_datasets]

"""Throughput of the device preprocessing / augmentation (csrc/prep_ops.hip)
beside the CPU restatement (oracle/prep.py, numpy + torch, one image at a time).

  preprocess: 64 decoded uint8 radiographs of 2048 x 1664 (MURA-like sizes) ->
              histogram equalisation, crop, pad, area resize to 512, normalise
  augment:    bs=256 uint8 [256,1,512,512] -> fp32 [256,3,512,512]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vlp_amd.augment import Augmenter, preprocess  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    g = np.random.default_rng(0)
    imgs = [g.integers(0, 256, (2048, 1664), dtype=np.uint8) for _ in range(64)]
    dev_imgs = [torch.from_numpy(i).cuda() for i in imgs]
    t = timed(lambda: preprocess(dev_imgs, 512, 127.5, 73.9, channels=3), 5)
    mpx = 64 * 2048 * 1664 / 1e6
    print(f"preprocess (device-resident input): {t * 1e3:.2f} ms / 64 images = {64 / t:.0f} images/s, "
          f"{mpx / t / 1e3:.1f} Gpx/s")
    t2 = timed(lambda: preprocess(imgs, 512, 127.5, 73.9, channels=3), 3)
    print(f"preprocess (host input incl. pinned upload): {t2 * 1e3:.2f} ms / 64 images = {64 / t2:.0f} images/s")
    x = torch.randint(0, 256, (256, 1, 512, 512), dtype=torch.uint8, device="cuda")
    a = Augmenter(seed=0)
    t3 = timed(lambda: a(x, channels=3, mean=127.5, std=73.9), 10)
    print(f"augment bs=256 512^2 u8 -> fp32 x3: {t3 * 1e3:.2f} ms = {256 / t3:.0f} images/s "
          f"({256 * 512 * 512 * (1 + 12) / t3 / 1e9:.0f} GB/s written+read)")
    try:
        import oracle.prep as op
        tc = time.perf_counter()
        for im in imgs[:2]:
            op.preprocess(im, 512, 127.5, 73.9, 3)
        tc = (time.perf_counter() - tc) / 2
        print(f"cpu restatement preprocess: {tc * 1e3:.0f} ms / image = {1 / tc:.1f} images/s (1 process)")
    except ImportError:
        pass


if __name__ == "__main__":
    main()

"""Epoch-end retrieval metrics at cache sizes of a real
epoch: precision@{3,5,10,15} over N image embeddings + image->text
recall@{3,5,10,15}, E = 128.  Times the module's GPU path (chunked fp32
similarity GEMM + vlp_row_topk) against the reference formulation (full N x N
matrix + torch.topk) on the same GPU, and reports the peak memory of each.
  python tools/retrieval_bench.py [--n 50000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
import torch  # noqa: E402


def reference_path(img, txt, lab, ks):
    """The reference's arithmetic (:364-439) with torch ops on the GPU."""
    e = torch.nn.functional.normalize(img)
    sim = e @ e.T
    p = {k: ((lab.unsqueeze(1) == lab[sim.topk(k + 1, dim=1).indices[:, 1:]]).sum(1).float() / k).mean().item()
         for k in ks}
    del sim
    i, t = torch.nn.functional.normalize(img), torch.nn.functional.normalize(txt)
    sim = i @ t.T
    tgt = torch.arange(i.shape[0], device=i.device)
    r = {k: (sim.topk(k, dim=1).indices == tgt.unsqueeze(1)).any(1).sum().item() / i.shape[0] for k in ks}
    return p, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    args = ap.parse_args()
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    N, E, ks = args.n, 128, [3, 5, 10, 15]
    img = torch.randn(N, E, device=dev)
    txt = img + 3.0 * torch.randn(N, E, device=dev)
    lab = torch.randint(0, 2, (N,), device=dev)
    m = VisionLanguageModule.__new__(VisionLanguageModule)
    res = {}
    for name, fn in (("hip_chunked", lambda: (VisionLanguageModule.precision_at_k_on_image_embeddings(m, img, lab, ks),
                                               VisionLanguageModule.recall_at_k_on_image_text_retreival(m, img, txt, ks))),
                     ("torch_full_matrix", lambda: reference_path(img, txt, lab, ks))):
        fn()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
        base = torch.cuda.memory_allocated(dev)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        res[name] = {"ms": round((time.perf_counter() - t0) * 1e3, 2),
                     "peak_extra_mb": round((torch.cuda.max_memory_allocated(dev) - base) / 1e6, 1),
                     "precision": out[0], "recall": out[1]}
    same = all(abs(res["hip_chunked"][m_][k] - res["torch_full_matrix"][m_][k]) < 1e-6
               for m_ in ("precision", "recall") for k in ks)
    print(json.dumps({"n": N, "e": E, "ks": ks, "results": res, "metrics_identical": same}))


if __name__ == "__main__":
    main()

"""Golden vectors for the late-fusion finetune loss, produced by
running the REFERENCE's own code in this container:
  * src/utils/coral_loss/coral.py `coral` (:5-15) and `compute_covariance` (:18-37);
  * src/models/baseline/FusionModule.py `_compute_loss` (:341-390), called unbound on
    a minimal `self` (label_weights, hparams.coral_lambda, device), so its BCE weighting
    and CORAL gating run as written.
Stand-ins (no arithmetic): lightning, torchmetrics.classification, timm, torchxrayvision
(FusionModule.py imports them at module level).
    python tests/golden/make_fusion_golden.py   -> tests/golden/fusion_loss.pt
"""
import os
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("VLP_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)

from tests.golden.make_golden import _install_stubs  # noqa: E402


def import_reference_fusion():
    _install_stubs()
    tmc = types.ModuleType("torchmetrics.classification")
    for n in ("BinaryAccuracy", "BinaryPrecision", "BinaryRecall", "BinaryF1Score", "BinaryAUROC"):
        setattr(tmc, n, type(n, (), {}))
    sys.modules["torchmetrics.classification"] = tmc
    sys.modules["torchmetrics"].classification = tmc
    sys.modules["torchxrayvision"] = types.ModuleType("torchxrayvision")
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        import src.models.baseline.FusionModule as fm
        import src.utils.coral_loss.coral as cr
    finally:
        os.chdir(cwd)
    return fm, cr


def main():
    fm, cr = import_reference_fusion()
    g = torch.Generator().manual_seed(11)
    out = {}
    # coral known answers, with gradients (autograd through the reference formula)
    cases = {"d512_5v7": (5, 7, 512), "d3_2v3": (2, 3, 3), "d1_4v3": (4, 3, 1), "d512_16v12": (16, 12, 512)}
    for name, (ns, nt, d) in cases.items():
        s = torch.randn(ns, d, generator=g, dtype=torch.float64).float().requires_grad_()
        t = (torch.randn(nt, d, generator=g, dtype=torch.float64) * 1.5 + 0.3).float().requires_grad_()
        loss = cr.coral(s, t)
        gs, gt = torch.autograd.grad(loss, (s, t))
        out[f"coral_{name}"] = {"source": s.detach(), "target": t.detach(), "loss": loss.detach(),
                                "grad_source": gs, "grad_target": gt}
    # the reference's own example rows (coral.py __main__): source vs the large-difference target
    src = torch.tensor([[1.0], [1.0], [1.1], [0.9]])
    tgt = torch.tensor([[10.0], [10.0], [11.0]])
    out["coral_example"] = {"source": src, "target": tgt, "loss": cr.coral(src, tgt)}

    # FusionModule._compute_loss, unbound, on synthetic features/logits
    def fake_self(lw, lam):
        return types.SimpleNamespace(label_weights=torch.tensor(lw),
                                     hparams=types.SimpleNamespace(coral_lambda=lam),
                                     device=torch.device("cpu"))
    loss_cases = []
    for B, lw, lam, ds in ((8, (1.0, 1.0), 0.0, None), (8, (0.7, 2.5), 0.5, None),
                           (6, (1.0, 3.0), 1.0, ["INTERNAL"] + ["BTXRD"] * 5),   # 1 internal: no coral
                           (16, (0.4, 1.6), 2.0, None)):
        feats = torch.randn(B, 512, 2, 2, generator=g, dtype=torch.float64).float()
        logits = torch.randn(B, generator=g, dtype=torch.float64).float()
        labels = torch.randint(0, 2, (B,), generator=g)
        if ds is None:
            ds = ["INTERNAL" if i % 2 == 0 else "BTXRD" for i in range(B)]
        f = feats.clone().requires_grad_()
        lg = logits.clone().requires_grad_()
        tot, cls, cor = fm.FusionModule._compute_loss(fake_self(lw, lam), f, lg, labels, ds)
        gf, gl = torch.autograd.grad(tot, (f, lg), allow_unused=True)
        loss_cases.append({"features": feats, "logits": logits, "labels": labels, "dataset": ds,
                           "label_weights": torch.tensor(lw), "coral_lambda": torch.tensor(lam),
                           "loss": tot.detach(), "classification_loss": cls.detach(),
                           "coral_loss": torch.as_tensor(cor).detach(),
                           "grad_features": gf if gf is not None else torch.zeros_like(feats),
                           "grad_logits": gl})
    out["compute_loss"] = loss_cases
    path = os.path.join(HERE, "fusion_loss.pt")
    torch.save(out, path)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

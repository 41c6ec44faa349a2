"""Imaging-only baseline (reference src/models/baseline/OnlyImagingModule.py).

CPU: the metric restatement against scikit-learn's accuracy / precision /
recall / F1 / ROC-AUC (torchmetrics' Binary* values at threshold 0.5); the
state-dict layout (timm resnet34(num_classes=1): trunk + fc 512->1); the
supported-model errors.  _compute_loss is FusionModule's, which
tests/test_fusion.py pins to the reference-run goldens.
GPU: the fp32 training step against a CPU oracle (oracle/resnet34.py trunk +
fc, weighted BCE + CORAL) on the same weights and batch for resnet34 and
nest_small (64^2, DropPath off); bf16 uint8 step, optimizer step and the
combined validation evaluation.
"""
import functools

import pytest
import torch
import torch.nn.functional as F

from oracle import weights as W
from oracle.fusion import coral as oracle_coral


def _labels_probs(n, seed):
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 2, (n,), generator=g)
    p = torch.rand(n, generator=g)
    p[:n // 4] = (p[:n // 4] * 4).round() / 4     # ties for the AUROC rank average
    return p, y


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_binary_metrics_vs_sklearn(seed):
    from sklearn.metrics import accuracy_score, f1_score, precision_score, recall_score, roc_auc_score
    from src.models.baseline.OnlyImagingModule import BinaryMetrics
    p, y = _labels_probs(97, seed)
    m = BinaryMetrics()
    m.update(p[:40], y[:40])
    m.update(p[40:], y[40:])
    r = m.compute()
    pred = (p >= 0.5).long().numpy()
    yn = y.numpy()
    assert abs(r["accuracy"] - accuracy_score(yn, pred)) < 1e-12
    assert abs(r["precision"] - precision_score(yn, pred, zero_division=0)) < 1e-12
    assert abs(r["recall"] - recall_score(yn, pred, zero_division=0)) < 1e-12
    assert abs(r["f1"] - f1_score(yn, pred, zero_division=0)) < 1e-12
    assert abs(r["auroc"] - roc_auc_score(yn, p.numpy())) < 1e-12
    # no predicted positives: precision / F1 are 0 (torchmetrics' zero_division)
    r0 = BinaryMetrics()
    r0.update(torch.zeros(4), torch.tensor([0, 1, 0, 1]))
    assert r0.compute()["precision"] == 0.0 and r0.compute()["f1"] == 0.0


def test_state_dict_and_model_errors():
    from oracle.resnet34 import ResNet34
    from src.models.baseline.OnlyImagingModule import OnlyImagingModule
    m = OnlyImagingModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), device="cpu")
    ref = {"network." + k for k in ResNet34().state_dict()} | {"network.fc.weight", "network.fc.bias"}
    assert set(m.state_dict()) == ref
    assert m.network.fc.weight.shape == (1, 512)
    assert sum(p.numel() for p in m.parameters()) == 21284672 + 513
    with pytest.raises(ValueError):
        OnlyImagingModule("alexnet", None, device="cpu")
    for name in ("resnet50", "vit_base_patch16_224", "resnet50-res512-all"):
        with pytest.raises(NotImplementedError):
            OnlyImagingModule(name, None, device="cpu")


def _batch(B, H, seed=0):
    g = torch.Generator().manual_seed(seed)
    x_u8 = torch.randint(0, 256, (B, 1, H, H), generator=g, dtype=torch.uint8)
    x = ((x_u8.float() - 127.5) / 73.9).repeat(1, 3, 1, 1)
    return {"x-ray": x, "x-ray-u8": x_u8, "tumor": torch.tensor([0, 1] * (B // 2)),
            "dataset": ["INTERNAL" if i % 3 else "BTXRD" for i in range(B)]}


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _oracle_loss(feat_map, logits, labels, dataset, lw, lam):
    w = torch.where(labels == 0, torch.tensor(lw[0]), torch.tensor(lw[1]))
    cls = F.binary_cross_entropy_with_logits(logits, labels.float(), weight=w)
    pooled = feat_map.mean((2, 3))
    mi = torch.tensor([d == "INTERNAL" for d in dataset])
    mb = torch.tensor([d == "BTXRD" for d in dataset])
    return cls + lam * oracle_coral(pooled[mi], pooled[mb])


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["resnet34", "nest_small"])
def test_step_vs_oracle_fp32(model):
    import oracle.nest as on
    from oracle.resnet34 import ResNet34
    from src.models.baseline.OnlyImagingModule import OnlyImagingModule
    lw, lam = (0.6, 2.5), 0.5
    B, H = 6, 64
    batch = _batch(B, H)
    torch.manual_seed(4)
    m = OnlyImagingModule(model, functools.partial(torch.optim.AdamW, lr=1e-3), label_weights=lw,
                          coral_lambda=lam, compute_dtype="fp32", image_size=H, drop_path_rate=0.0)
    if model == "resnet34":
        trunk = ResNet34()
        sd = {k: W.value_for("image_encoder.model." + k, v.shape, 4).to(v.dtype) for k, v in trunk.state_dict().items()}
        trunk.load_state_dict(sd)
        head = torch.nn.Linear(512, 1)
        m.network.load_state_dict({**sd, "fc.weight": head.weight.detach(), "fc.bias": head.bias.detach()})
    else:
        trunk = on.nest_small(img_size=H, drop_path_rate=0.0)
        trunk.load_state_dict({k: v.detach().cpu() for k, v in m.network.state_dict().items()
                               if not k.startswith("head.")})
        head = torch.nn.Linear(384, 1)
        head.load_state_dict({"weight": m.network.head.weight.detach().cpu(),
                              "bias": m.network.head.bias.detach().cpu()})
    m.train()
    trunk.train()
    if model == "nest_small":
        for lvl in trunk.levels:
            for layer in lvl.transformer_encoder:
                layer.drop_path = 0.0
    f = trunk.forward_features(batch["x-ray"])
    lo = head(f.mean((2, 3))).flatten()
    Lo = _oracle_loss(f, lo, batch["tumor"], batch["dataset"], lw, lam)
    Lo.backward()
    loss = m.training_step(batch)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - Lo.item()) < 1e-4, (loss.item(), Lo.item())
    assert float(m.logged["train/coral_loss"].detach()) > 0.0
    og = {("network." + k): p.grad for k, p in trunk.named_parameters()}
    og.update({"network." + ("fc" if model == "resnet34" else "head") + "." + k: p.grad
               for k, p in head.named_parameters()})
    worst = max((_rel(p.grad, og[k]), k) for k, p in m.named_parameters()
                if og.get(k) is not None and og[k].norm() > 1e-6)
    assert worst[0] < 1e-3, worst


@pytest.mark.gpu
def test_bf16_u8_step_and_validation_epoch():
    from src.models.baseline.OnlyImagingModule import OnlyImagingModule
    B, H = 8, 64
    batch = _batch(B, H, seed=3)
    torch.manual_seed(5)
    m32 = OnlyImagingModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), coral_lambda=0.5,
                            compute_dtype="fp32")
    m16 = OnlyImagingModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), coral_lambda=0.5,
                            compute_dtype="bf16")
    m16.load_state_dict(m32.state_dict())
    l32 = m32.training_step(batch).item()
    opt = m16.configure_optimizers()["optimizer"]
    w0 = m16.network.conv1.weight.detach().clone()
    loss = m16.training_step({k: v for k, v in batch.items() if k != "x-ray"})
    loss.backward()
    opt.step()
    assert abs(loss.item() - l32) < 5e-2, (loss.item(), l32)
    assert not torch.equal(w0, m16.network.conv1.weight.detach())
    m16.on_train_epoch_end()
    assert 0.0 <= m16.logged["train/auroc"] <= 1.0
    # validation over two dataloaders, then the combined evaluation
    m16.eval()
    m16.validation_step(batch, 0, 0)
    m16.validation_step(_batch(B, H, seed=4), 0, 1)
    with pytest.raises(ValueError):
        m16.validation_step(batch, 0, 2)
    m16.on_validation_epoch_end()
    for k in ("loss", "classification_loss", "coral_loss", "accuracy", "precision", "recall", "f1", "auroc"):
        assert f"val/combined/{k}" in m16.logged, k
    assert "val/internal/auroc" in m16.logged and "val/btxrd/loss" in m16.logged
    assert m16.all_val_probs == []

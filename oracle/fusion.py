"""ORACLE (test infrastructure): CPU fp32 restatement of the reference's late-fusion
finetune step, SURVEY §8(f) row 1.  Only tests/ may import this.

References (src/models/baseline/FusionModule.py, src/utils/coral_loss/coral.py):
  * image_network = timm resnet34 with num_classes=10 (:91-93): forward_features ->
    [B,512,h,w], forward_head = global average pool + fc 512->10 (timm ResNet);
  * tabular_network (:60-70): Linear(15,32) BN1d ReLU Linear(32,20) BN1d ReLU
    Linear(20,10) BN1d ReLU over cat(anatomy_site[9], age[4], sex[2]) (:322);
  * combination_network Linear(20,1) over cat(image_logits, clinical_logits), flattened (:117, :324);
  * _compute_loss (:341-390): BCE-with-logits with per-sample weights
    label_weights[label]; CORAL (coral.py:5-37) between the spatially averaged
    features of the "INTERNAL" and "BTXRD" samples, times coral_lambda, only when
    coral_lambda != 0 and each domain has >= 2 samples in the batch.
The CORAL arithmetic below follows coral.py's formula (ones-row column sums,
mean outer product, d_t_d, / (n-1); squared Frobenius difference / (4 d^2)).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle.resnet34 import ResNet34


def covariance(x):                       # coral.py:23-37
    n = x.shape[0]
    col_sum = torch.ones(1, n, dtype=x.dtype) @ x
    mean = col_sum / n
    return (x.t() @ x - mean.t() @ mean) * (1.0 / (n - 1))


def coral(source, target):               # coral.py:5-15
    d = source.shape[1]
    diff = covariance(source) - covariance(target)
    return (diff * diff).sum() / (4 * d * d)


class _Classifier(nn.Module):
    """timm resnet34(num_classes=10): conv trunk + avg pool + fc."""

    def __init__(self):
        super().__init__()
        self.trunk = ResNet34()
        self.fc = nn.Linear(512, 10)

    def forward_features(self, x):
        return self.trunk.forward_features(x)

    def forward_head(self, f):
        return self.fc(f.mean((2, 3)) if f.dim() == 4 else f)


class OracleFusion(nn.Module):
    def __init__(self, label_weights=(1.0, 1.0), coral_lambda=0.0):
        super().__init__()
        self.tabular_network = nn.Sequential(
            nn.Linear(15, 32), nn.BatchNorm1d(32), nn.ReLU(),
            nn.Linear(32, 20), nn.BatchNorm1d(20), nn.ReLU(),
            nn.Linear(20, 10), nn.BatchNorm1d(10), nn.ReLU())
        self.image_network = _Classifier()
        self.combination_network = nn.Linear(20, 1)
        self.label_weights = torch.tensor(label_weights)
        self.coral_lambda = coral_lambda

    def forward(self, x, age, sex, site):
        f = self.image_network.forward_features(x)
        img_logits = self.image_network.forward_head(f)
        clin = self.tabular_network(torch.cat((site, age, sex), dim=1))
        return self.combination_network(torch.cat((img_logits, clin), dim=1)).flatten(), f

    def compute_loss(self, f, logits, labels, dataset):
        w = torch.where(labels == 0, self.label_weights[0], self.label_weights[1]).to(logits.dtype)
        # labels in the logits' dtype (float() in the reference; the fp64 envelope runs this in double)
        cls = F.binary_cross_entropy_with_logits(logits, labels.to(logits.dtype), weight=w)
        if self.coral_lambda == 0.0:
            return cls, cls, torch.tensor(0.0)
        pooled = f.mean((2, 3)) if f.dim() == 4 else f
        mi = torch.tensor([d == "INTERNAL" for d in dataset])
        mb = torch.tensor([d == "BTXRD" for d in dataset])
        if mi.sum() <= 1 or mb.sum() <= 1:
            return cls, cls, torch.tensor(0.0)
        c = self.coral_lambda * coral(pooled[mi], pooled[mb])
        return cls + c, cls, c

    def state_dict_hip_layout(self):
        """Keys as the reference FusionModule holds them (image_network.<timm>)."""
        out = {}
        for k, v in self.state_dict().items():
            out[k.replace("image_network.trunk.", "image_network.")] = v
        return out

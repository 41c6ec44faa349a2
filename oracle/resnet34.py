"""ORACLE (test infrastructure): timm `resnet34` restated in plain torch.

Reference call site: src/models/pretrain/VisionLanguageModule.py:27-35
    timm.create_model(model, pretrained=False, num_classes=0, global_pool="avg", drop_rate=...)
timm==1.0.15 (environment.yaml:327) is not installed and not vendored, so this
restates its published architecture: conv1 7x7/2 (3->64, pad 3, no bias) -> bn1
-> relu -> maxpool 3x3/2 pad 1 -> layer1..4 of BasicBlocks [3,4,6,3] at widths
[64,128,256,512] (3x3 convs, BN, ReLU; 1x1/2 conv + BN downsample on the first
block of layers 2-4) -> global average pool -> dropout(drop_rate) -> [B, 512].
State-dict keys follow timm exactly (conv1, bn1, layerX.Y.{conv1,bn1,conv2,bn2,
downsample.0,downsample.1}), which is what the reference's checkpoints and the
finetuning consumers (OnlyImagingModule.py:76-80) rely on.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        shortcut = x
        x = F.relu(self.bn1(self.conv1(x)))
        x = self.bn2(self.conv2(x))
        if self.downsample is not None:
            shortcut = self.downsample(shortcut)
        return F.relu(x + shortcut)


class ResNet34(nn.Module):
    LAYERS = (3, 4, 6, 3)
    WIDTHS = (64, 128, 256, 512)

    def __init__(self, drop_rate: float = 0.0, zero_init_last: bool = True):
        super().__init__()
        self.drop_rate = drop_rate
        self.num_features = 512
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        inplanes = 64
        for li, (n, planes) in enumerate(zip(self.LAYERS, self.WIDTHS)):
            stride = 1 if li == 0 else 2
            blocks = []
            for b in range(n):
                s = stride if b == 0 else 1
                ds = None
                if b == 0 and (s != 1 or inplanes != planes):
                    ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, s, bias=False),
                                       nn.BatchNorm2d(planes))
                blocks.append(BasicBlock(inplanes, planes, s, ds))
                inplanes = planes
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        # timm ResNet.init_weights: kaiming_normal(fan_out, relu) convs, BN 1/0,
        # zero_init_last -> every BasicBlock's bn2.weight = 0
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_last:
            for m in self.modules():
                if isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def forward_features(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        return self.layer4(x)

    def forward(self, x):
        x = self.forward_features(x).mean((2, 3))
        if self.drop_rate > 0.0:
            x = F.dropout(x, p=self.drop_rate, training=self.training)
        return x


def create_model(name, pretrained=False, num_classes=0, global_pool="avg", drop_rate=0.0, **kw):
    """Stand-in for timm.create_model for the one architecture on the hot path."""
    if name != "resnet34" or num_classes != 0 or global_pool != "avg" or pretrained:
        raise ValueError(f"oracle only restates resnet34 feature extraction, got {name}")
    return ResNet34(drop_rate=drop_rate)

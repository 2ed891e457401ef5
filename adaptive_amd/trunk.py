"""ResNet-152 convolutional trunk: ``AttentiveCNN.resnet_conv``.

The reference builds it as ``nn.Sequential(*list(torchvision.models.resnet152(pretrained=True)
.children())[:-2])`` (``code_src/models/baseline_attention.py:16-18``) and runs it on every batch
(``:43``).  torchvision is not part of this image, and the pretrained weights cannot be fetched
offline, so this module rebuilds the same network with the same child order and parameter names —
``0`` conv1, ``1`` bn1, ``2`` relu, ``3`` maxpool, ``4``-``7`` layer1-4 of Bottleneck blocks
[3, 8, 36, 3] with the stride on the 3x3 convolution — so a reference checkpoint's
``encoder.resnet_conv.*`` tensors load into it unchanged, and random-inits it the way torchvision
does (He-normal fan-out convolutions, unit BatchNorm).

Compute runs on PyTorch-ROCm (MIOpen convolutions, fp32 as in the reference): the trunk is not part
of the decode hot path (it runs once per image, before the decode), so it is the library path
here, not a hand-written kernel.  ``fold_bn()`` returns an inference copy with every BatchNorm folded
into its convolution (one conv + bias per layer, channels-last), which is what ``sampler`` uses in
eval mode.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn

LAYERS_152 = (3, 8, 36, 3)


class Bottleneck(nn.Module):
    """torchvision Bottleneck (expansion 4): 1x1 -> 3x3 (stride) -> 1x1, identity or downsample."""

    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


def _layer(inplanes: int, planes: int, blocks: int, stride: int):
    down = None
    if stride != 1 or inplanes != planes * 4:
        down = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False), nn.BatchNorm2d(planes * 4))
    mods = [Bottleneck(inplanes, planes, stride, down)]
    mods += [Bottleneck(planes * 4, planes) for _ in range(1, blocks)]
    return nn.Sequential(*mods)


def resnet_conv(layers=LAYERS_152) -> nn.Sequential:
    """``list(resnet152().children())[:-2]`` as an ``nn.Sequential``: images [B,3,224,224] ->
    A [B,2048,7,7]."""
    mods = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, stride=2, padding=1)]
    inplanes = 64
    for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
        mods.append(_layer(inplanes, planes, n, 1 if i == 0 else 2))
        inplanes = planes * 4
    seq = nn.Sequential(*mods)
    for m in seq.modules():  # torchvision's ResNet init
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
    return seq


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    """conv followed by eval-mode BN -> one conv with bias: w' = w g / sqrt(var + eps),
    b' = beta - mean g / sqrt(var + eps)."""
    f = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding, bias=True)
    with torch.no_grad():
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        f.weight.copy_(conv.weight * scale.view(-1, 1, 1, 1))
        f.bias.copy_(bn.bias - bn.running_mean * scale)
    return f.to(conv.weight.device)


class _FoldedBottleneck(nn.Module):
    def __init__(self, blk: Bottleneck):
        super().__init__()
        self.c1 = _fold(blk.conv1, blk.bn1)
        self.c2 = _fold(blk.conv2, blk.bn2)
        self.c3 = _fold(blk.conv3, blk.bn3)
        self.down = None if blk.downsample is None else _fold(blk.downsample[0], blk.downsample[1])

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        out = torch.relu(self.c1(x))
        out = torch.relu(self.c2(out))
        return torch.relu(self.c3(out) + idt)


def fold_bn(seq: nn.Sequential) -> nn.Sequential:
    """Inference copy of a ``resnet_conv`` with BatchNorm folded into the convolutions (eval-mode
    semantics: running statistics), in channels-last memory format for MIOpen's NHWC kernels."""
    stem = nn.Sequential(_fold(seq[0], seq[1]), nn.ReLU(inplace=True), copy.deepcopy(seq[3]))
    blocks = [_FoldedBottleneck(b) for layer in list(seq)[4:] for b in layer]
    out = nn.Sequential(stem, *blocks).eval()
    return out.to(memory_format=torch.channels_last)

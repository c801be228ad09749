"""ResNet-50 (BASELINE configs 2, 3, 5: collective ResNet-50 on 1 / 8 MI355X,
elastic ResNet-50) — written out here because torchvision is not part of the
image.  Standard v1.5 bottleneck architecture (stride on the 3×3 conv).

MI355X choices: channels_last bf16 activations; every convolution on
hand-written kernels — the 7×7 stem as a space-to-depth 4×4 convolution over a
16-channel image (ops._StemFn), the rest on the NHWC implicit GEMM
(csrc/hip/conv.hip: BatchNorm forward statistics from its epilogue, the previous
BatchNorm's backward statistics from its input-gradient epilogue) or, per
product where measured faster, the token-major GEMMs (gemm_nt4 / gemm_dw4) for
the wide 1×1 stride-1 products; the residual branch's gradient summed inside
conv1's input-gradient epilogue;
BatchNorm (fp32 statistics and affine params) fused with ReLU and the residual
add into HIP kernels (ops.bn_act); parameters live in a flat fp32 arena
(parallel.flat) so the gradient all-reduce buckets are slices.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.downsample = downsample

    def forward(self, x):
        # every convolution + BatchNorm (+ ReLU, + residual add) through
        # ops.conv_bn_act: hand-written kernels per product (NHWC implicit GEMM
        # with the BatchNorm statistics in its epilogue, or the token-major GEMMs
        # for the wide 1×1 products), BN apply fused with ReLU / residual.
        # conv1 forks x for the identity / downsample branch: that branch's
        # gradient joins conv1's dX in the dX kernel's epilogue.
        out, xa = ops.conv_bn_act(self.conv1, self.bn1, x, fork=True)
        out = ops.conv_bn_act(self.conv2, self.bn2, out)
        if self.downsample is not None:
            # bn3 and the downsample BatchNorm in one apply pass where fused
            return ops.conv_bn_ds_act(self.conv3, self.bn3, out, self.downsample[0], self.downsample[1], xa)
        return ops.conv_bn_act(self.conv3, self.bn3, out, relu=True, residual=xa)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, width=64):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        cin = width
        stages = []
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                ds = None
                if j == 0 and (stride != 1 or cin != w * Bottleneck.expansion):
                    ds = nn.Sequential(nn.Conv2d(cin, w * Bottleneck.expansion, 1, stride=stride, bias=False),
                                       nn.BatchNorm2d(w * Bottleneck.expansion))
                blocks.append(Bottleneck(cin, w, stride if j == 0 else 1, ds))
                cin = w * Bottleneck.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():  # zero-init last BN of each block (standard large-batch recipe)
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.bn3.weight)

    def forward(self, x):
        # the space-to-depth stem with BatchNorm + ReLU + max-pool fused on the HIP path
        x = ops.conv_bn_relu_maxpool(self.conv1, self.bn1, x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = ops.global_avg_pool(x)  # its backward writes the channels_last gradient directly (HIP path)
        return self.fc(x)


def resnet50(num_classes=1000):
    return ResNet((3, 4, 6, 3), num_classes)


def resnet18_like_tiny(num_classes=10):
    """Tiny variant for CPU tests."""
    return ResNet((1, 1, 1, 1), num_classes, width=8)

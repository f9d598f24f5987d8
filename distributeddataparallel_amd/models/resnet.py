"""ResNet family (torchvision-identical structure, random init).

The reference trains ``torchvision.models.resnet18`` with its ``fc`` replaced by
``Linear(512, 10)`` (``ref:dpp.py:11-18``); BASELINE.json's headline config is ResNet-50.
torchvision is not installed here, so the architectures are rebuilt layer-for-layer
(parameter counts match torchvision: ResNet-50 = 25,557,032; ResNet-18/10-class =
11,181,642 — SURVEY.md Appendix A). ``norm_layer`` lets the bench swap in xddp's fused
HIP BatchNorm(+ReLU) without changing the parameter/buffer layout or state_dict keys.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional, Type, Union

import torch
import torch.nn as nn

__all__ = ["ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "SimpleCNN"]


def conv3x3(i, o, stride=1, groups=1, dilation=1):
    return nn.Conv2d(i, o, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, 1, stride=stride, bias=False)


def _conv_bn_fusion() -> bool:
    """XDDP_CONV_BN_FUSION=0 turns off the 1x1-conv + BN-statistics fusion (A/B switch)."""
    import os

    return os.environ.get("XDDP_CONV_BN_FUSION", "1") != "0"


def _stem_fusion() -> bool:
    """XDDP_STEM_FUSION=0 runs the stem's bn1 -> ReLU -> maxpool as separate kernels (A/B switch)."""
    import os

    return os.environ.get("XDDP_STEM_FUSION", "1") != "0"


def _ds_link() -> bool:
    """XDDP_CONV_EPI_DS=0 keeps the stride-2 downsample's input gradient out of the next conv1's
    epilogue (scattered to full resolution and reduced by the producer instead; A/B switch)."""
    import os

    return os.environ.get("XDDP_CONV_EPI_DS", "1") != "0"


# Set by ResNet.forward while its fused blocks may hand a pending output (ops/conv_bn.py
# PendingApply) to the next block: only inside the model's own forward, where the next block's
# conv1 is that output's first reader and the final output is resolved before it leaves.
_PEND = threading.local()


def _pending_ok() -> bool:
    return getattr(_PEND, "on", False)


def _ds_defer() -> bool:
    """XDDP_DS_DEFER=0 keeps the downsample's own BN apply pass (A/B switch): by default the block's
    final apply pass applies it to the raw downsample output on the fly."""
    import os

    return os.environ.get("XDDP_DS_DEFER", "1") != "0"


def _bn_relu(norm_layer, c):
    """Return (bn, act). A fused norm layer (``fuses_relu``) absorbs the ReLU."""
    bn = norm_layer(c)
    if getattr(bn, "fuses_relu", False):
        bn.relu = True
        return bn, nn.Identity()
    return bn, nn.ReLU(inplace=True)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1, self.act1 = _bn_relu(norm_layer, planes)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self._fused_add = getattr(self.bn2, "supports_add_relu", False)

    def forward(self, x):
        x, xr = x if isinstance(x, tuple) else (x, x)  # (main, residual-path alias) from a fused producer
        identity = xr if self.downsample is None else self.downsample(xr)
        out = self.act1(self.bn1(self.conv1(x)))
        out = self.conv2(out)
        if self._fused_add:
            return self.bn2(out, residual=identity, relu=True, dual_output=True)
        out = self.bn2(out)
        out += identity
        return self.relu(out)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1, self.act1 = _bn_relu(norm_layer, width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2, self.act2 = _bn_relu(norm_layer, width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self._fused_add = getattr(self.bn3, "supports_add_relu", False)

    def forward(self, x):
        x, xr = x if isinstance(x, tuple) else (x, x)  # (main, residual-path alias) from a fused producer
        if self._fused_add and _conv_bn_fusion() and self.training:
            # 1x1 convs with the BN statistics in the conv's MFMA epilogue (ops/conv_bn.py)
            from ..ops.conv_bn import conv1x1_bn_act, conv3x3_bn_relu

            # previous block's output consumed by conv1 and the identity (or the stride-2
            # downsample): their backward hands that gradient to conv1's input-gradient GEMM
            # epilogue (ops/conv_bn.py:EpiLink)
            link = getattr(x, "_xddp_epi", None)
            ds = self.downsample
            if ds is not None and not (ds[0].stride[0] == 2 and _ds_link()):
                link = None
            # the downsample's BN apply is folded into the final apply pass (ops/conv_bn.py:DeferredBN)
            defer = _ds_defer()
            if ds is not None and link is None:
                identity = conv1x1_bn_act(xr, ds[0], ds[1], defer=defer)
            out = conv1x1_bn_act(x, self.conv1, self.bn1, relu=True, link_x=link)
            # BN2's apply happens in conv3's GEMM prologue (ops/conv_bn.py:PendingApply) — only
            # inside ResNet.forward with no hook anywhere in the blocks (a hook on act2 would
            # otherwise see a tensor conv3's prologue has not written yet)
            out = self.act2(conv3x3_bn_relu(out, self.conv2, self.bn2, pending=_pending_ok()))
            if ds is None:
                identity = xr
            elif link is not None:  # issued after conv2: its backward runs before conv1's
                identity = conv1x1_bn_act(xr, ds[0], ds[1], link_ds=link, defer=defer)
            # the block output's apply (BN3 + identity + ReLU) happens in the next block's conv1
            # GEMM prologue when ResNet.forward allows it
            return conv1x1_bn_act(out, self.conv3, self.bn3, residual=identity, relu=True, dual_output=True,
                                  link_res=link if ds is None else None, pending=_pending_ok())
        identity = xr if self.downsample is None else self.downsample(xr)
        out = self.act1(self.bn1(self.conv1(x)))
        out = self.act2(self.bn2(self.conv2(out)))
        out = self.conv3(out)
        if self._fused_add:
            return self.bn3(out, residual=identity, relu=True, dual_output=True)
        out = self.bn3(out)
        out += identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, groups: int = 1, width_per_group: int = 64,
                 norm_layer: Optional[Callable[..., nn.Module]] = None,
                 pool_layer: Optional[Callable[..., nn.Module]] = None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        if pool_layer is None:
            if getattr(norm_layer, "fuses_relu", False):  # the fused-kernel stack: native NHWC max-pool too
                from ..ops.pool import FusedMaxPool2d

                pool_layer = FusedMaxPool2d
            else:
                pool_layer = nn.MaxPool2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1, self.relu = _bn_relu(norm_layer, self.inplanes)
        self.maxpool = pool_layer(kernel_size=3, stride=2, padding=1)
        if hasattr(self.maxpool, "dual_output"):
            self.maxpool.dual_output = True
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif hasattr(m, "weight") and hasattr(m, "running_mean") and m.weight is not None:
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, self.dilation,
                        norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                dilation=self.dilation, norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def _no_block_hooks(self) -> bool:
        """No forward hook can see a pending tensor (a block output, or BN2's output inside a block,
        must not be read before the consuming conv's prologue writes it): none on the layers, any
        module inside their blocks (act2 included), or globally."""
        from torch.nn.modules import module as _mod

        if _mod._global_forward_hooks or _mod._global_forward_pre_hooks:
            return False
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for m in layer.modules():
                if m._forward_hooks or m._forward_pre_hooks:
                    return False
        return True

    def forward(self, x):
        fused = (getattr(self.bn1, "fuses_relu", False) and getattr(self.bn1, "relu", False)
                 and getattr(self.maxpool, "dual_output", None) is not None and self.training and _stem_fusion())
        pooled = None
        if fused:
            from ..ops.stem import resnet_stem, stem_supported

            if stem_supported(x, self.conv1, self.bn1, self.maxpool):
                # conv (BN statistics in its epilogue) -> normalize/ReLU/pool: ops/stem.py
                pooled = resnet_stem(x, self.conv1, self.bn1, self.maxpool, dual=self.maxpool.dual_output)
        if pooled is None:
            x = self.conv1(x)
            if fused:
                # bn1 -> ReLU -> maxpool without the normalized activation in HBM (ops/pool.py)
                from ..ops.pool import stem_bn_relu_maxpool

                pooled = stem_bn_relu_maxpool(x, self.bn1, self.maxpool, dual=self.maxpool.dual_output)
        x = pooled if pooled is not None else self.maxpool(self.relu(self.bn1(x)))
        prev = _pending_ok()
        _PEND.on = fused and self._no_block_hooks()
        try:
            x = self.layer1(x)
            x = self.layer2(x)
            x = self.layer3(x)
            x = self.layer4(x)
        finally:
            _PEND.on = prev
        if isinstance(x, tuple):  # fused blocks hand (output, alias) to the next block
            x = x[0]
        if fused:
            from ..ops.conv_bn import resolve

            resolve(x)  # the last block's output has no conv1 to absorb its apply
        if fused and isinstance(self.avgpool, nn.AdaptiveAvgPool2d) and self.avgpool.output_size in (1, (1, 1)):
            from ..ops.pool import global_avg_pool

            x = global_avg_pool(x)  # channels_last gradient without a transpose copy
        else:
            x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)


class SimpleCNN(nn.Module):
    """The reference's model wrapper (``ref:dpp.py:11-18``): ResNet-18 with a 10-class head.

    Random init instead of ImageNet weights (no network; quirk Q3). state_dict keys match the
    reference (``model.conv1.weight`` ... ; ``module.model.*`` once wrapped in DDP).
    """

    def __init__(self, num_classes: int = 10, norm_layer=None):
        super().__init__()
        self.model = resnet18(norm_layer=norm_layer)
        self.model.fc = nn.Linear(512, num_classes)

    def forward(self, x):
        return self.model(x)

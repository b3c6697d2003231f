"""ResNet / ResNeXt / Wide-ResNet (reference: python/paddle/vision/models/resnet.py).

Same module structure and parameter names as the reference (conv1/bn1/layer1..4/fc,
BottleneckBlock.conv1..3/bn1..3/downsample). Adds ``data_format``: "NHWC" keeps
every activation channels-last, the layout MI355X conv/BN kernels run fastest in
(the reference is NCHW-only here).
"""
from __future__ import annotations

from ... import nn
from ...nn import functional as F
from ...nn.layer.conv_norm_pool import _BatchNormBase
from ...tensor import flatten
from ...ops import conv_gemm as _conv_gemm


def _bn_act(bn, x, residual=None, relu=True):
    """bn(x) (+ residual) (+ relu) as ONE fused pass when ``bn`` is a plain BatchNorm layer
    (the reference's fuse_bn_add_act_ops pass, done eagerly); otherwise the unfused ops."""
    from ...framework.core import _mode
    # static Programs (jit.save / to_static) record the reference's separate batch_norm /
    # elementwise_add / relu ops — what a saved inference model holds
    if type(bn) in (nn.BatchNorm2D, nn.BatchNorm) and getattr(bn, "_act", None) is None and not _mode.static:
        return F.batch_norm_act(x, bn._mean, bn._variance, bn.weight, bn.bias, bn.training, bn._momentum,
                                bn._epsilon, bn._data_format, bn._use_global_stats, residual=residual,
                                act="relu" if relu else None)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y

__all__ = ["ResNet", "BasicBlock", "BottleneckBlock", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "resnext50_32x4d", "resnext50_64x4d", "resnext101_32x4d", "resnext101_64x4d", "resnext152_32x4d",
           "resnext152_64x4d", "wide_resnet50_2", "wide_resnet101_2"]


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(planes, data_format=data_format)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(planes, data_format=data_format)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = _bn_act(self.bn1, self.conv1(x))
        if self.downsample is not None:
            identity = self.downsample(x)
        return _bn_act(self.bn2, self.conv2(out), residual=identity)


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(width, data_format=data_format)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups, dilation=dilation,
                               bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(width, data_format=data_format)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=data_format)
        self.bn3 = norm_layer(planes * self.expansion, data_format=data_format)
        self.relu = nn.ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        # conv1 adds x's other gradient in its dgrad epilogue (conv_gemm.res_route_begin): the residual
        # gradient of an identity block, the shortcut conv's dx of a downsample block
        route = _conv_gemm.res_route_begin(x._t, "bn" if self.downsample is None else "conv") if self.training \
            else None
        try:
            out = _bn_act(self.bn1, self.conv1(x))
            out = _bn_act(self.bn2, self.conv2(out))
            if self.downsample is not None:
                identity = self.downsample(x)
            return _bn_act(self.bn3, self.conv3(out), residual=identity)
        finally:
            _conv_gemm.res_route_end(x._t, route)


class ResNet(nn.Layer):
    _DEPTH = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}

    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1, data_format="NCHW"):
        super().__init__()
        layers = self._DEPTH[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        self._norm_layer = nn.BatchNorm2D
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False, data_format=data_format)
        self.bn1 = self._norm_layer(self.inplanes, data_format=data_format)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(kernel_size=3, stride=2, padding=1, data_format=data_format)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=data_format)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride, bias_attr=False,
                          data_format=self.data_format),
                norm_layer(planes * block.expansion, data_format=self.data_format))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, previous_dilation,
                        norm_layer, data_format=self.data_format)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                norm_layer=norm_layer, data_format=self.data_format))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_bn_act(self.bn1, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = flatten(x, 1)
            x = self.fc(x)
        return x


def _resnet(arch, Block, depth, pretrained, **kwargs):
    if pretrained:
        raise RuntimeError("pretrained weights are not available offline; load a .pdparams with set_state_dict")
    return ResNet(Block, depth, **kwargs)


def resnet18(pretrained=False, **kwargs):
    return _resnet("resnet18", BasicBlock, 18, pretrained, **kwargs)


def resnet34(pretrained=False, **kwargs):
    return _resnet("resnet34", BasicBlock, 34, pretrained, **kwargs)


def resnet50(pretrained=False, **kwargs):
    return _resnet("resnet50", BottleneckBlock, 50, pretrained, **kwargs)


def resnet101(pretrained=False, **kwargs):
    return _resnet("resnet101", BottleneckBlock, 101, pretrained, **kwargs)


def resnet152(pretrained=False, **kwargs):
    return _resnet("resnet152", BottleneckBlock, 152, pretrained, **kwargs)


def resnext50_32x4d(pretrained=False, **kwargs):
    return _resnet("resnext50_32x4d", BottleneckBlock, 50, pretrained, groups=32, width=4, **kwargs)


def resnext50_64x4d(pretrained=False, **kwargs):
    return _resnet("resnext50_64x4d", BottleneckBlock, 50, pretrained, groups=64, width=4, **kwargs)


def resnext101_32x4d(pretrained=False, **kwargs):
    return _resnet("resnext101_32x4d", BottleneckBlock, 101, pretrained, groups=32, width=4, **kwargs)


def resnext101_64x4d(pretrained=False, **kwargs):
    return _resnet("resnext101_64x4d", BottleneckBlock, 101, pretrained, groups=64, width=4, **kwargs)


def resnext152_32x4d(pretrained=False, **kwargs):
    return _resnet("resnext152_32x4d", BottleneckBlock, 152, pretrained, groups=32, width=4, **kwargs)


def resnext152_64x4d(pretrained=False, **kwargs):
    return _resnet("resnext152_64x4d", BottleneckBlock, 152, pretrained, groups=64, width=4, **kwargs)


def wide_resnet50_2(pretrained=False, **kwargs):
    return _resnet("wide_resnet50_2", BottleneckBlock, 50, pretrained, width=64 * 2, **kwargs)


def wide_resnet101_2(pretrained=False, **kwargs):
    return _resnet("wide_resnet101_2", BottleneckBlock, 101, pretrained, width=64 * 2, **kwargs)

"""Classic CNN families (reference: python/paddle/vision/models/{lenet,alexnet,vgg,mobilenetv1,
mobilenetv2,mobilenetv3,shufflenetv2,squeezenet,densenet,googlenet,inceptionv3}.py).
Architectures follow the original papers with the reference's constructor signatures."""
from __future__ import annotations

import math

from ... import nn
from ...nn import functional as F
from ...tensor import flatten, concat, reshape, transpose, split

__all__ = ["LeNet", "AlexNet", "alexnet", "VGG", "vgg11", "vgg13", "vgg16", "vgg19", "MobileNetV1", "mobilenet_v1",
           "MobileNetV2", "mobilenet_v2", "MobileNetV3Small", "MobileNetV3Large", "mobilenet_v3_small",
           "mobilenet_v3_large", "ShuffleNetV2", "shufflenet_v2_x0_25", "shufflenet_v2_x0_33", "shufflenet_v2_x0_5",
           "shufflenet_v2_x1_0", "shufflenet_v2_x1_5", "shufflenet_v2_x2_0", "shufflenet_v2_swish", "SqueezeNet",
           "squeezenet1_0", "squeezenet1_1", "DenseNet", "densenet121", "densenet161", "densenet169", "densenet201",
           "densenet264", "GoogLeNet", "googlenet", "InceptionV3", "inception_v3"]


def _no_pretrained(pretrained):
    if pretrained:
        raise RuntimeError("pretrained weights are not available offline; load a .pdparams with set_state_dict")


# ---------------------------------------------------------------------------- LeNet
class LeNet(nn.Layer):
    def __init__(self, num_classes=10):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(nn.Conv2D(1, 6, 3, stride=1, padding=1), nn.ReLU(), nn.MaxPool2D(2, 2),
                                      nn.Conv2D(6, 16, 5, stride=1, padding=0), nn.ReLU(), nn.MaxPool2D(2, 2))
        if num_classes > 0:
            self.fc = nn.Sequential(nn.Linear(400, 120), nn.Linear(120, 84), nn.Linear(84, num_classes))

    def forward(self, inputs):
        x = self.features(inputs)
        if self.num_classes > 0:
            x = flatten(x, 1)
            x = self.fc(x)
        return x


# ---------------------------------------------------------------------------- AlexNet
class AlexNet(nn.Layer):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.num_classes = num_classes
        self._conv1 = nn.Conv2D(3, 64, 11, stride=4, padding=5)
        self._conv2 = nn.Conv2D(64, 192, 5, padding=2)
        self._conv3 = nn.Conv2D(192, 384, 3, padding=1)
        self._conv4 = nn.Conv2D(384, 256, 3, padding=1)
        self._conv5 = nn.Conv2D(256, 256, 3, padding=1)
        self._pool = nn.MaxPool2D(3, 2)
        self._relu = nn.ReLU()
        if num_classes > 0:
            self._drop1 = nn.Dropout(0.5)
            self._fc6 = nn.Linear(256 * 6 * 6, 4096)
            self._drop2 = nn.Dropout(0.5)
            self._fc7 = nn.Linear(4096, 4096)
            self._fc8 = nn.Linear(4096, num_classes)

    def forward(self, x):
        x = self._pool(self._relu(self._conv1(x)))
        x = self._pool(self._relu(self._conv2(x)))
        x = self._relu(self._conv3(x))
        x = self._relu(self._conv4(x))
        x = self._pool(self._relu(self._conv5(x)))
        x = F.adaptive_avg_pool2d(x, (6, 6))
        if self.num_classes > 0:
            x = flatten(x, 1)
            x = self._relu(self._fc6(self._drop1(x)))
            x = self._relu(self._fc7(self._drop2(x)))
            x = self._fc8(x)
        return x


def alexnet(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return AlexNet(**kwargs)


# ---------------------------------------------------------------------------- VGG
class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True):
        super().__init__()
        self.features = features
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(), nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


_VGG_CFG = {"A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
            "B": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
            "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
            "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]}


def _vgg_features(cfg, batch_norm=False):
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2D(2, 2))
        else:
            layers.append(nn.Conv2D(c, v, 3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v))
            layers.append(nn.ReLU())
            c = v
    return nn.Sequential(*layers)


def _vgg(cfg, pretrained, batch_norm, **kwargs):
    _no_pretrained(pretrained)
    return VGG(_vgg_features(_VGG_CFG[cfg], batch_norm), **kwargs)


def vgg11(pretrained=False, batch_norm=False, **kwargs):
    return _vgg("A", pretrained, batch_norm, **kwargs)


def vgg13(pretrained=False, batch_norm=False, **kwargs):
    return _vgg("B", pretrained, batch_norm, **kwargs)


def vgg16(pretrained=False, batch_norm=False, **kwargs):
    return _vgg("D", pretrained, batch_norm, **kwargs)


def vgg19(pretrained=False, batch_norm=False, **kwargs):
    return _vgg("E", pretrained, batch_norm, **kwargs)


# ---------------------------------------------------------------------------- MobileNets
class ConvBNLayer(nn.Layer):
    def __init__(self, in_c, out_c, k, stride=1, padding=0, groups=1, act="relu"):
        super().__init__()
        self._conv = nn.Conv2D(in_c, out_c, k, stride=stride, padding=padding, groups=groups, bias_attr=False)
        self._norm_layer = nn.BatchNorm2D(out_c)
        self._act = act

    def forward(self, x):
        x = self._norm_layer(self._conv(x))
        if self._act == "relu":
            x = F.relu(x)
        elif self._act == "relu6":
            x = F.relu6(x)
        elif self._act == "hardswish":
            x = F.hardswish(x)
        elif self._act == "swish":
            x = F.swish(x)
        return x


class DepthwiseSeparable(nn.Layer):
    def __init__(self, in_c, out_c1, out_c2, num_groups, stride, scale):
        super().__init__()
        self._depthwise_conv = ConvBNLayer(in_c, int(out_c1 * scale), 3, stride, 1, int(num_groups * scale))
        self._pointwise_conv = ConvBNLayer(int(out_c1 * scale), int(out_c2 * scale), 1)

    def forward(self, x):
        return self._pointwise_conv(self._depthwise_conv(x))


class MobileNetV1(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.scale, self.num_classes, self.with_pool = scale, num_classes, with_pool
        self.conv1 = ConvBNLayer(3, int(32 * scale), 3, 2, 1)
        cfg = [(32, 32, 64, 32, 1), (64, 64, 128, 64, 2), (128, 128, 128, 128, 1), (128, 128, 256, 128, 2),
               (256, 256, 256, 256, 1), (256, 256, 512, 256, 2)] + [(512, 512, 512, 512, 1)] * 5 + \
              [(512, 512, 1024, 512, 2), (1024, 1024, 1024, 1024, 1)]
        self.dwsl = nn.Sequential(*[DepthwiseSeparable(int(a * scale), b, c, d, s, scale) for a, b, c, d, s in cfg])
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(int(1024 * scale), num_classes)

    def forward(self, x):
        x = self.dwsl(self.conv1(x))
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.fc(flatten(x, 1))
        return x


def mobilenet_v1(pretrained=False, scale=1.0, **kwargs):
    _no_pretrained(pretrained)
    return MobileNetV1(scale=scale, **kwargs)


def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class InvertedResidual(nn.Layer):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNLayer(inp, hidden, 1, act="relu6"))
        layers += [ConvBNLayer(hidden, hidden, 3, stride, 1, groups=hidden, act="relu6"),
                   nn.Conv2D(hidden, oup, 1, bias_attr=False), nn.BatchNorm2D(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        input_channel = _make_divisible(32 * scale)
        self.last_channel = _make_divisible(1280 * max(1.0, scale))
        cfg = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2], [6, 320, 1, 1]]
        features = [ConvBNLayer(3, input_channel, 3, 2, 1, act="relu6")]
        for t, c, n, s in cfg:
            out = _make_divisible(c * scale)
            for i in range(n):
                features.append(InvertedResidual(input_channel, out, s if i == 0 else 1, t))
                input_channel = out
        features.append(ConvBNLayer(input_channel, self.last_channel, 1, act="relu6"))
        self.features = nn.Sequential(*features)
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last_channel, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


def mobilenet_v2(pretrained=False, scale=1.0, **kwargs):
    _no_pretrained(pretrained)
    return MobileNetV2(scale=scale, **kwargs)


class SqueezeExcitation(nn.Layer):
    def __init__(self, c, squeeze):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2D(1)
        self.fc1 = nn.Conv2D(c, squeeze, 1)
        self.fc2 = nn.Conv2D(squeeze, c, 1)

    def forward(self, x):
        s = F.hardsigmoid(self.fc2(F.relu(self.fc1(self.avgpool(x)))), slope=0.2, offset=0.5)
        return x * s


class InvertedResidualV3(nn.Layer):
    def __init__(self, in_c, exp, out_c, k, stride, use_se, act):
        super().__init__()
        self.use_res = stride == 1 and in_c == out_c
        self.expand = in_c != exp
        if self.expand:
            self.expand_conv = ConvBNLayer(in_c, exp, 1, act=act)
        self.bottleneck_conv = ConvBNLayer(exp, exp, k, stride, (k - 1) // 2, groups=exp, act=act)
        self.use_se = use_se
        if use_se:
            self.mid_se = SqueezeExcitation(exp, _make_divisible(exp // 4))
        self.linear_conv = ConvBNLayer(exp, out_c, 1, act=None)

    def forward(self, x):
        y = self.expand_conv(x) if self.expand else x
        y = self.bottleneck_conv(y)
        if self.use_se:
            y = self.mid_se(y)
        y = self.linear_conv(y)
        return x + y if self.use_res else y


class _MobileNetV3(nn.Layer):
    def __init__(self, cfg, last_channel, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        firstc = _make_divisible(16 * scale)
        self.conv = ConvBNLayer(3, firstc, 3, 2, 1, act="hardswish")
        blocks = []
        c = firstc
        for k, exp, out, se, act, s in cfg:
            e = _make_divisible(exp * scale)
            o = _make_divisible(out * scale)
            blocks.append(InvertedResidualV3(c, e, o, k, s, se, act))
            c = o
        self.blocks = nn.Sequential(*blocks)
        self.lastconv = ConvBNLayer(c, 6 * c, 1, act="hardswish")
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(6 * c, last_channel), nn.Hardswish(), nn.Dropout(0.2),
                                            nn.Linear(last_channel, num_classes))

    def forward(self, x):
        x = self.lastconv(self.blocks(self.conv(x)))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


class MobileNetV3Small(_MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        cfg = [(3, 16, 16, True, "relu", 2), (3, 72, 24, False, "relu", 2), (3, 88, 24, False, "relu", 1),
               (5, 96, 40, True, "hardswish", 2), (5, 240, 40, True, "hardswish", 1), (5, 240, 40, True, "hardswish", 1),
               (5, 120, 48, True, "hardswish", 1), (5, 144, 48, True, "hardswish", 1), (5, 288, 96, True, "hardswish", 2),
               (5, 576, 96, True, "hardswish", 1), (5, 576, 96, True, "hardswish", 1)]
        super().__init__(cfg, _make_divisible(1024 * scale), scale, num_classes, with_pool)


class MobileNetV3Large(_MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        cfg = [(3, 16, 16, False, "relu", 1), (3, 64, 24, False, "relu", 2), (3, 72, 24, False, "relu", 1),
               (5, 72, 40, True, "relu", 2), (5, 120, 40, True, "relu", 1), (5, 120, 40, True, "relu", 1),
               (3, 240, 80, False, "hardswish", 2), (3, 200, 80, False, "hardswish", 1), (3, 184, 80, False, "hardswish", 1),
               (3, 184, 80, False, "hardswish", 1), (3, 480, 112, True, "hardswish", 1), (3, 672, 112, True, "hardswish", 1),
               (5, 672, 160, True, "hardswish", 2), (5, 960, 160, True, "hardswish", 1), (5, 960, 160, True, "hardswish", 1)]
        super().__init__(cfg, _make_divisible(1280 * scale), scale, num_classes, with_pool)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kwargs):
    _no_pretrained(pretrained)
    return MobileNetV3Small(scale=scale, **kwargs)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kwargs):
    _no_pretrained(pretrained)
    return MobileNetV3Large(scale=scale, **kwargs)


# ---------------------------------------------------------------------------- ShuffleNetV2
def _channel_shuffle(x, groups):
    return F.channel_shuffle(x, groups)


class ShuffleUnit(nn.Layer):
    def __init__(self, in_c, out_c, stride, act):
        super().__init__()
        self.stride = stride
        branch = out_c // 2
        if stride == 2:
            self._conv_dw_1 = ConvBNLayer(in_c, in_c, 3, 2, 1, groups=in_c, act=None)
            self._conv_linear_1 = ConvBNLayer(in_c, branch, 1, act=act)
            in2 = in_c
        else:
            in2 = branch
        self._conv_pw_2 = ConvBNLayer(in2, branch, 1, act=act)
        self._conv_dw_2 = ConvBNLayer(branch, branch, 3, stride, 1, groups=branch, act=None)
        self._conv_linear_2 = ConvBNLayer(branch, branch, 1, act=act)

    def forward(self, x):
        if self.stride == 1:
            x1, x2 = split(x, 2, axis=1)
        else:
            x1 = self._conv_linear_1(self._conv_dw_1(x))
            x2 = x
        x2 = self._conv_linear_2(self._conv_dw_2(self._conv_pw_2(x2)))
        return _channel_shuffle(concat([x1, x2], axis=1), 2)


class ShuffleNetV2(nn.Layer):
    _CH = {0.25: [-1, 24, 24, 48, 96, 512], 0.33: [-1, 24, 32, 64, 128, 512], 0.5: [-1, 24, 48, 96, 192, 1024],
           1.0: [-1, 24, 116, 232, 464, 1024], 1.5: [-1, 24, 176, 352, 704, 1024], 2.0: [-1, 24, 224, 488, 976, 2048]}

    def __init__(self, scale=1.0, act="relu", num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        stage_out = self._CH[scale]
        self._conv1 = ConvBNLayer(3, stage_out[1], 3, 2, 1, act=act)
        self._max_pool = nn.MaxPool2D(3, 2, 1)
        blocks = []
        for i, rep in enumerate([4, 8, 4]):
            for j in range(rep):
                blocks.append(ShuffleUnit(stage_out[i + 1] if j == 0 else stage_out[i + 2], stage_out[i + 2],
                                          2 if j == 0 else 1, act))
        self._block_list = nn.Sequential(*blocks)
        self._last_conv = ConvBNLayer(stage_out[-2], stage_out[-1], 1, act=act)
        if with_pool:
            self._pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self._fc = nn.Linear(stage_out[-1], num_classes)

    def forward(self, x):
        x = self._last_conv(self._block_list(self._max_pool(self._conv1(x))))
        if self.with_pool:
            x = self._pool2d_avg(x)
        if self.num_classes > 0:
            x = self._fc(flatten(x, 1))
        return x


def _shuffle(scale, act="relu", pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return ShuffleNetV2(scale=scale, act=act, **kwargs)


def shufflenet_v2_x0_25(pretrained=False, **kwargs):
    return _shuffle(0.25, pretrained=pretrained, **kwargs)


def shufflenet_v2_x0_33(pretrained=False, **kwargs):
    return _shuffle(0.33, pretrained=pretrained, **kwargs)


def shufflenet_v2_x0_5(pretrained=False, **kwargs):
    return _shuffle(0.5, pretrained=pretrained, **kwargs)


def shufflenet_v2_x1_0(pretrained=False, **kwargs):
    return _shuffle(1.0, pretrained=pretrained, **kwargs)


def shufflenet_v2_x1_5(pretrained=False, **kwargs):
    return _shuffle(1.5, pretrained=pretrained, **kwargs)


def shufflenet_v2_x2_0(pretrained=False, **kwargs):
    return _shuffle(2.0, pretrained=pretrained, **kwargs)


def shufflenet_v2_swish(pretrained=False, **kwargs):
    return _shuffle(1.0, act="swish", pretrained=pretrained, **kwargs)


# ---------------------------------------------------------------------------- SqueezeNet
class MakeFire(nn.Layer):
    def __init__(self, in_c, squeeze, e1, e3):
        super().__init__()
        self._conv = nn.Conv2D(in_c, squeeze, 1)
        self._conv_path1 = nn.Conv2D(squeeze, e1, 1)
        self._conv_path2 = nn.Conv2D(squeeze, e3, 3, padding=1)

    def forward(self, x):
        x = F.relu(self._conv(x))
        return concat([F.relu(self._conv_path1(x)), F.relu(self._conv_path2(x))], axis=1)


class SqueezeNet(nn.Layer):
    def __init__(self, version, num_classes=1000, with_pool=True):
        super().__init__()
        self.version, self.num_classes, self.with_pool = version, num_classes, with_pool
        if version == "1.0":
            self._conv = nn.Conv2D(3, 96, 7, stride=2)
            fires = [(96, 16, 64, 64), (128, 16, 64, 64), (128, 32, 128, 128), "M", (256, 32, 128, 128),
                     (256, 48, 192, 192), (384, 48, 192, 192), (384, 64, 256, 256), "M", (512, 64, 256, 256)]
        else:
            self._conv = nn.Conv2D(3, 64, 3, stride=2, padding=1)
            fires = [(64, 16, 64, 64), (128, 16, 64, 64), "M", (128, 32, 128, 128), (256, 32, 128, 128), "M",
                     (256, 48, 192, 192), (384, 48, 192, 192), (384, 64, 256, 256), (512, 64, 256, 256)]
        self._pool = nn.MaxPool2D(3, 2)
        seq = []
        for f in fires:
            seq.append(nn.MaxPool2D(3, 2) if f == "M" else MakeFire(*f))
        self._fires = nn.Sequential(*seq)
        self._drop = nn.Dropout(0.5)
        if num_classes > 0:
            self._conv9 = nn.Conv2D(512, num_classes, 1)
        if with_pool:
            self._avg_pool = nn.AdaptiveAvgPool2D(1)

    def forward(self, x):
        x = self._pool(F.relu(self._conv(x)))
        x = self._fires(x)
        x = self._drop(x)
        if self.num_classes > 0:
            x = F.relu(self._conv9(x))
        if self.with_pool:
            x = self._avg_pool(x)
            x = flatten(x, 1)
        return x


def squeezenet1_0(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return SqueezeNet("1.0", **kwargs)


def squeezenet1_1(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return SqueezeNet("1.1", **kwargs)


# ---------------------------------------------------------------------------- DenseNet
class DenseLayer(nn.Layer):
    def __init__(self, in_c, growth, bn_size, dropout):
        super().__init__()
        self.bn1 = nn.BatchNorm2D(in_c)
        self.conv1 = nn.Conv2D(in_c, bn_size * growth, 1, bias_attr=False)
        self.bn2 = nn.BatchNorm2D(bn_size * growth)
        self.conv2 = nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False)
        self.dropout = dropout

    def forward(self, x):
        y = self.conv1(F.relu(self.bn1(x)))
        y = self.conv2(F.relu(self.bn2(y)))
        if self.dropout:
            y = F.dropout(y, self.dropout, training=self.training)
        return concat([x, y], axis=1)


class DenseNet(nn.Layer):
    _CFG = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]), 169: (64, 32, [6, 12, 32, 32]),
            201: (64, 32, [6, 12, 48, 32]), 264: (64, 32, [6, 12, 64, 48])}

    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        init_c, growth, blocks = self._CFG[layers]
        self.conv1 = nn.Conv2D(3, init_c, 7, stride=2, padding=3, bias_attr=False)
        self.bn1 = nn.BatchNorm2D(init_c)
        self.pool1 = nn.MaxPool2D(3, 2, 1)
        feats = []
        c = init_c
        for i, n in enumerate(blocks):
            for _ in range(n):
                feats.append(DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                feats += [nn.BatchNorm2D(c), nn.ReLU(), nn.Conv2D(c, c // 2, 1, bias_attr=False), nn.AvgPool2D(2, 2)]
                c //= 2
        self.dense_blocks = nn.Sequential(*feats)
        self.batch_norm = nn.BatchNorm2D(c)
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.out = nn.Linear(c, num_classes)

    def forward(self, x):
        x = self.pool1(F.relu(self.bn1(self.conv1(x))))
        x = F.relu(self.batch_norm(self.dense_blocks(x)))
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.out(flatten(x, 1))
        return x


def _densenet(layers, pretrained, **kwargs):
    _no_pretrained(pretrained)
    return DenseNet(layers=layers, **kwargs)


def densenet121(pretrained=False, **kwargs):
    return _densenet(121, pretrained, **kwargs)


def densenet161(pretrained=False, **kwargs):
    return _densenet(161, pretrained, **kwargs)


def densenet169(pretrained=False, **kwargs):
    return _densenet(169, pretrained, **kwargs)


def densenet201(pretrained=False, **kwargs):
    return _densenet(201, pretrained, **kwargs)


def densenet264(pretrained=False, **kwargs):
    return _densenet(264, pretrained, **kwargs)


# ---------------------------------------------------------------------------- GoogLeNet
class Inception(nn.Layer):
    def __init__(self, in_c, c1, c3r, c3, c5r, c5, pp):
        super().__init__()
        self._conv1 = ConvBNLayer(in_c, c1, 1)
        self._conv3r = ConvBNLayer(in_c, c3r, 1)
        self._conv3 = ConvBNLayer(c3r, c3, 3, padding=1)
        self._conv5r = ConvBNLayer(in_c, c5r, 1)
        self._conv5 = ConvBNLayer(c5r, c5, 5, padding=2)
        self._pool = nn.MaxPool2D(3, 1, 1)
        self._convprj = ConvBNLayer(in_c, pp, 1)

    def forward(self, x):
        return concat([self._conv1(x), self._conv3(self._conv3r(x)), self._conv5(self._conv5r(x)),
                       self._convprj(self._pool(x))], axis=1)


class GoogLeNet(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self._conv = ConvBNLayer(3, 64, 7, 2, 3)
        self._pool = nn.MaxPool2D(3, 2, 1)
        self._conv_1 = ConvBNLayer(64, 64, 1)
        self._conv_2 = ConvBNLayer(64, 192, 3, padding=1)
        self._ince3a = Inception(192, 64, 96, 128, 16, 32, 32)
        self._ince3b = Inception(256, 128, 128, 192, 32, 96, 64)
        self._ince4a = Inception(480, 192, 96, 208, 16, 48, 64)
        self._ince4b = Inception(512, 160, 112, 224, 24, 64, 64)
        self._ince4c = Inception(512, 128, 128, 256, 24, 64, 64)
        self._ince4d = Inception(512, 112, 144, 288, 32, 64, 64)
        self._ince4e = Inception(528, 256, 160, 320, 32, 128, 128)
        self._ince5a = Inception(832, 256, 160, 320, 32, 128, 128)
        self._ince5b = Inception(832, 384, 192, 384, 48, 128, 128)
        if with_pool:
            self._pool_5 = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self._drop = nn.Dropout(0.4)
            self._fc_out = nn.Linear(1024, num_classes)
            self._pool_o1 = nn.AdaptiveAvgPool2D(3)
            self._conv_o1 = ConvBNLayer(512, 128, 1)
            self._fc_o1 = nn.Linear(1152, 1024)
            self._drop_o1 = nn.Dropout(0.7)
            self._out1 = nn.Linear(1024, num_classes)
            self._pool_o2 = nn.AdaptiveAvgPool2D(3)
            self._conv_o2 = ConvBNLayer(528, 128, 1)
            self._fc_o2 = nn.Linear(1152, 1024)
            self._drop_o2 = nn.Dropout(0.7)
            self._out2 = nn.Linear(1024, num_classes)

    def forward(self, x):
        x = self._pool(self._conv(x))
        x = self._pool(self._conv_2(self._conv_1(x)))
        x = self._pool(self._ince3b(self._ince3a(x)))
        ince4a = self._ince4a(x)
        x = self._ince4c(self._ince4b(ince4a))
        ince4d = self._ince4d(x)
        x = self._pool(self._ince4e(ince4d))
        x = self._ince5b(self._ince5a(x))
        if self.with_pool:
            x = self._pool_5(x)
        if self.num_classes > 0:
            out = self._fc_out(self._drop(flatten(x, 1)))
            o1 = flatten(self._conv_o1(self._pool_o1(ince4a)), 1)
            out1 = self._out1(self._drop_o1(F.relu(self._fc_o1(o1))))
            o2 = flatten(self._conv_o2(self._pool_o2(ince4d)), 1)
            out2 = self._out2(self._drop_o2(F.relu(self._fc_o2(o2))))
            return [out, out1, out2]
        return x


def googlenet(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return GoogLeNet(**kwargs)


# ---------------------------------------------------------------------------- InceptionV3
class _IncA(nn.Layer):
    def __init__(self, c, pf):
        super().__init__()
        self.b1 = ConvBNLayer(c, 64, 1)
        self.b5_1 = ConvBNLayer(c, 48, 1)
        self.b5_2 = ConvBNLayer(48, 64, 5, padding=2)
        self.b3_1 = ConvBNLayer(c, 64, 1)
        self.b3_2 = ConvBNLayer(64, 96, 3, padding=1)
        self.b3_3 = ConvBNLayer(96, 96, 3, padding=1)
        self.bp = ConvBNLayer(c, pf, 1)

    def forward(self, x):
        return concat([self.b1(x), self.b5_2(self.b5_1(x)), self.b3_3(self.b3_2(self.b3_1(x))),
                       self.bp(F.avg_pool2d(x, 3, 1, 1))], axis=1)


class _IncB(nn.Layer):
    def __init__(self, c):
        super().__init__()
        self.b3 = ConvBNLayer(c, 384, 3, 2)
        self.bd_1 = ConvBNLayer(c, 64, 1)
        self.bd_2 = ConvBNLayer(64, 96, 3, padding=1)
        self.bd_3 = ConvBNLayer(96, 96, 3, 2)

    def forward(self, x):
        return concat([self.b3(x), self.bd_3(self.bd_2(self.bd_1(x))), F.max_pool2d(x, 3, 2)], axis=1)


class _IncC(nn.Layer):
    def __init__(self, c, c7):
        super().__init__()
        self.b1 = ConvBNLayer(c, 192, 1)
        self.b7 = nn.Sequential(ConvBNLayer(c, c7, 1), ConvBNLayer(c7, c7, (1, 7), padding=(0, 3)),
                                ConvBNLayer(c7, 192, (7, 1), padding=(3, 0)))
        self.b7d = nn.Sequential(ConvBNLayer(c, c7, 1), ConvBNLayer(c7, c7, (7, 1), padding=(3, 0)),
                                 ConvBNLayer(c7, c7, (1, 7), padding=(0, 3)), ConvBNLayer(c7, c7, (7, 1), padding=(3, 0)),
                                 ConvBNLayer(c7, 192, (1, 7), padding=(0, 3)))
        self.bp = ConvBNLayer(c, 192, 1)

    def forward(self, x):
        return concat([self.b1(x), self.b7(x), self.b7d(x), self.bp(F.avg_pool2d(x, 3, 1, 1))], axis=1)


class _IncD(nn.Layer):
    def __init__(self, c):
        super().__init__()
        self.b3 = nn.Sequential(ConvBNLayer(c, 192, 1), ConvBNLayer(192, 320, 3, 2))
        self.b7 = nn.Sequential(ConvBNLayer(c, 192, 1), ConvBNLayer(192, 192, (1, 7), padding=(0, 3)),
                                ConvBNLayer(192, 192, (7, 1), padding=(3, 0)), ConvBNLayer(192, 192, 3, 2))

    def forward(self, x):
        return concat([self.b3(x), self.b7(x), F.max_pool2d(x, 3, 2)], axis=1)


class _IncE(nn.Layer):
    def __init__(self, c):
        super().__init__()
        self.b1 = ConvBNLayer(c, 320, 1)
        self.b3_1 = ConvBNLayer(c, 384, 1)
        self.b3_2a = ConvBNLayer(384, 384, (1, 3), padding=(0, 1))
        self.b3_2b = ConvBNLayer(384, 384, (3, 1), padding=(1, 0))
        self.bd_1 = ConvBNLayer(c, 448, 1)
        self.bd_2 = ConvBNLayer(448, 384, 3, padding=1)
        self.bd_3a = ConvBNLayer(384, 384, (1, 3), padding=(0, 1))
        self.bd_3b = ConvBNLayer(384, 384, (3, 1), padding=(1, 0))
        self.bp = ConvBNLayer(c, 192, 1)

    def forward(self, x):
        a = self.b3_1(x)
        d = self.bd_2(self.bd_1(x))
        return concat([self.b1(x), self.b3_2a(a), self.b3_2b(a), self.bd_3a(d), self.bd_3b(d),
                       self.bp(F.avg_pool2d(x, 3, 1, 1))], axis=1)


class InceptionV3(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.inception_stem = nn.Sequential(ConvBNLayer(3, 32, 3, 2), ConvBNLayer(32, 32, 3), ConvBNLayer(32, 64, 3, padding=1),
                                            nn.MaxPool2D(3, 2), ConvBNLayer(64, 80, 1), ConvBNLayer(80, 192, 3),
                                            nn.MaxPool2D(3, 2))
        self.inception_block_list = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64), _IncB(288),
                                                  _IncC(768, 128), _IncC(768, 160), _IncC(768, 160), _IncC(768, 192),
                                                  _IncD(768), _IncE(1280), _IncE(2048))
        if with_pool:
            self.avg_pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.2)
            self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.inception_block_list(self.inception_stem(x))
        if self.with_pool:
            x = self.avg_pool(x)
        if self.num_classes > 0:
            x = self.fc(self.dropout(flatten(x, 1)))
        return x


def inception_v3(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return InceptionV3(**kwargs)

"""Full-precision networks of the reference's model zoo (models/*.py), plain PyTorch.

Out of the hot path: they only provide the layer shapes and the block structure that
QuantModel rewraps (the attribute names -- conv1/bn1/relu1/.../downsample, conv[i],
use_res_connect, expand_ratio -- are the ones quant_block.py reads).  Weights are random
(kaiming / normal init); there is no network access for pretrained checkpoints.
"""
import math

import torch
import torch.nn as nn


# ------------------------------------------------------------------ ResNet (models/resnet.py)
def _conv3x3(cin, cout, stride=1, groups=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, groups=groups, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.relu2 = nn.ReLU(inplace=True)
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu1(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu2(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu3 = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu1(self.bn1(self.conv1(x)))
        out = self.relu2(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu3(out + identity)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


# ------------------------------------------------------------------ MobileNetV2 (models/mobilenetv2.py)
class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = round(inp * expand_ratio)
        self.stride = stride
        self.use_res_connect = stride == 1 and inp == oup
        self.expand_ratio = expand_ratio
        dw = [nn.Conv2d(hidden, hidden, 3, stride, 1, groups=hidden, bias=False),
              nn.BatchNorm2d(hidden), nn.ReLU6(inplace=True)]
        pw_lin = [nn.Conv2d(hidden, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)]
        if expand_ratio == 1:
            self.conv = nn.Sequential(*dw, *pw_lin)
        else:
            pw = [nn.Conv2d(inp, hidden, 1, 1, 0, bias=False), nn.BatchNorm2d(hidden),
                  nn.ReLU6(inplace=True)]
            self.conv = nn.Sequential(*pw, *dw, *pw_lin)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Module):
    SETTING = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1],
               [6, 160, 3, 2], [6, 320, 1, 1]]

    def __init__(self, n_class=1000, width_mult=1.0, dropout=0.0):
        super().__init__()
        cin = int(32 * width_mult)
        self.last_channel = int(1280 * width_mult) if width_mult > 1.0 else 1280
        feats = [nn.Sequential(nn.Conv2d(3, cin, 3, 2, 1, bias=False), nn.BatchNorm2d(cin),
                               nn.ReLU6(inplace=True))]
        for t, c, n, s in self.SETTING:
            cout = int(c * width_mult)
            for i in range(n):
                feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        feats.append(nn.Sequential(nn.Conv2d(cin, self.last_channel, 1, 1, 0, bias=False),
                                   nn.BatchNorm2d(self.last_channel), nn.ReLU6(inplace=True)))
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(dropout), nn.Linear(self.last_channel, n_class))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()

    def forward(self, x):
        return self.classifier(self.features(x).mean([2, 3]))


def mobilenetv2(**kw):
    return MobileNetV2(**kw)


# ------------------------------------------------------------------ RegNetX (models/regnet.py)
# The RegNet design space (Radosavovic et al. 2020): per-block widths u_j = w0 + wa*j are
# snapped to w0 * wm^round(log(u_j/w0)/log(wm)), rounded to multiples of 8, grouped into
# stages of equal width, then made compatible with the group width (bottleneck ratio 1).
# Module names follow the reference (f.a/a_bn/a_relu, f.b, f.c, proj/bn, relu) so the
# quant block mapping (QuantResBottleneckBlock) applies unchanged.
REGNETX = {"regnetx_200m": (36.44, 24, 2.49, 13, 8), "regnetx_400m": (24.48, 24, 2.54, 22, 16),
           "regnetx_600m": (36.97, 48, 2.24, 16, 24), "regnetx_800m": (35.73, 56, 2.28, 16, 16),
           "regnetx_1600m": (34.01, 80, 2.25, 18, 24), "regnetx_3200m": (26.31, 88, 2.25, 25, 48),
           "regnetx_4000m": (38.65, 96, 2.43, 23, 40), "regnetx_6400m": (60.83, 184, 2.07, 17, 56)}


def regnet_stages(wa, w0, wm, depth, gw, q=8):
    """(stage widths, stage depths, group widths) of a RegNetX configuration."""
    widths = []
    for j in range(depth):
        k = round(math.log((w0 + wa * j) / w0) / math.log(wm))
        widths.append(int(round(w0 * wm ** k / q) * q))
    sw, sd = [], []
    for w in widths:
        if sw and sw[-1] == w:
            sd[-1] += 1
        else:
            sw.append(w)
            sd.append(1)
    gs = [min(gw, w) for w in sw]
    sw = [int(round(w / g) * g) for w, g in zip(sw, gs)]
    return sw, sd, gs


class _BottleneckTransform(nn.Module):
    def __init__(self, w_in, w_out, stride, gw):
        super().__init__()
        self.a = nn.Conv2d(w_in, w_out, 1, 1, 0, bias=False)
        self.a_bn = nn.BatchNorm2d(w_out)
        self.a_relu = nn.ReLU(inplace=True)
        self.b = nn.Conv2d(w_out, w_out, 3, stride, 1, groups=w_out // gw, bias=False)
        self.b_bn = nn.BatchNorm2d(w_out)
        self.b_relu = nn.ReLU(inplace=True)
        self.c = nn.Conv2d(w_out, w_out, 1, 1, 0, bias=False)
        self.c_bn = nn.BatchNorm2d(w_out)

    def forward(self, x):
        for m in self.children():
            x = m(x)
        return x


class ResBottleneckBlock(nn.Module):
    def __init__(self, w_in, w_out, stride, gw):
        super().__init__()
        self.proj_block = w_in != w_out or stride != 1
        if self.proj_block:
            self.proj = nn.Conv2d(w_in, w_out, 1, stride, 0, bias=False)
            self.bn = nn.BatchNorm2d(w_out)
        self.f = _BottleneckTransform(w_in, w_out, stride, gw)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        skip = self.bn(self.proj(x)) if self.proj_block else x
        return self.relu(skip + self.f(x))


class RegNet(nn.Module):
    def __init__(self, wa, w0, wm, depth, gw, num_classes=1000, stem_w=32):
        super().__init__()
        sw, sd, gs = regnet_stages(wa, w0, wm, depth, gw)
        self.stem = nn.Sequential(nn.Conv2d(3, stem_w, 3, 2, 1, bias=False), nn.BatchNorm2d(stem_w),
                                  nn.ReLU(inplace=True))
        prev = stem_w
        for i, (w, d, g) in enumerate(zip(sw, sd, gs)):
            stage = nn.Sequential()
            for k in range(d):
                stage.add_module(f"b{k + 1}", ResBottleneckBlock(prev if k == 0 else w, w,
                                                                 2 if k == 0 else 1, g))
            self.add_module(f"s{i + 1}", stage)
            prev = w
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(prev, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0.0, math.sqrt(2.0 / fan_out))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 1.0 / float(m.weight.size(1)))
                m.bias.data.zero_()
        self.stages = len(sw)

    def forward(self, x):
        x = self.stem(x)
        for i in range(self.stages):
            x = getattr(self, f"s{i + 1}")(x)
        return self.fc(torch.flatten(self.avgpool(x), 1))


def _regnet(name):
    def build(**kw):
        return RegNet(*REGNETX[name], **kw)
    build.__name__ = name
    return build


ARCHS = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50,
         "mobilenetv2": mobilenetv2}
ARCHS.update({name: _regnet(name) for name in REGNETX})

"""BN folding (reference: quant/fold_bn.py).  One-shot host preprocessing with plain
PyTorch ops (out of the hot path): W' = W * g/sqrt(var+eps), b' = beta - g*mean/sqrt(var+eps)
(+ g*b/sqrt(var+eps) when the conv has a bias), then the BN becomes an identity."""
import torch
import torch.nn as nn


class StraightThrough(nn.Module):
    def forward(self, input):
        return input


def _fold_bn(conv_module, bn_module):
    w = conv_module.weight.data
    std = torch.sqrt(bn_module.running_var + bn_module.eps)
    shape = (conv_module.out_channels, 1, 1, 1) if w.dim() == 4 else (-1, 1)
    if bn_module.affine:
        weight = w * (bn_module.weight / std).view(shape)
        beta = bn_module.bias - bn_module.weight * bn_module.running_mean / std
        bias = beta if conv_module.bias is None else bn_module.weight * conv_module.bias / std + beta
    else:
        weight = w / std.view(shape)
        beta = -bn_module.running_mean / std
        bias = beta if conv_module.bias is None else conv_module.bias / std + beta
    return weight, bias


def fold_bn_into_conv(conv_module, bn_module):
    w, b = _fold_bn(conv_module, bn_module)
    if conv_module.bias is None:
        conv_module.bias = nn.Parameter(b)
    else:
        conv_module.bias.data = b
    conv_module.weight.data = w
    bn_module.running_mean = bn_module.bias.data
    bn_module.running_var = bn_module.weight.data ** 2


def reset_bn(module: nn.BatchNorm2d):
    if module.track_running_stats:
        module.running_mean.zero_()
        module.running_var.fill_(1 - module.eps)
    if module.affine:
        nn.init.ones_(module.weight)
        nn.init.zeros_(module.bias)


def is_bn(m):
    return isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d))


def is_absorbing(m):
    return isinstance(m, (nn.Conv2d, nn.Linear))


def search_fold_and_remove_bn(model):
    """fold_bn.py:67-79: fold every BN that directly follows a conv/linear sibling."""
    model.eval()
    prev = None
    for n, m in model.named_children():
        if is_bn(m) and is_absorbing(prev):
            fold_bn_into_conv(prev, m)
            setattr(model, n, StraightThrough())
        elif is_absorbing(m):
            prev = m
        else:
            prev = search_fold_and_remove_bn(m)
    return prev


def search_fold_and_reset_bn(model):
    model.eval()
    prev = None
    for n, m in model.named_children():
        if is_bn(m) and is_absorbing(prev):
            fold_bn_into_conv(prev, m)
        else:
            search_fold_and_reset_bn(m)
        prev = m

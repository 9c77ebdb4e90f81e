"""Real-shape parity cases (BASELINE configs 2-5): one block of each network at its real
channel counts, seeded so that the reference side (make_golden.py, CPU) and the test side
(tests/test_realshape_gpu.py) build bit-identical FP weights and calibration inputs
without shipping them -- the fixtures hold only what the reference computed from them.

Torch's CPU randn / kaiming_normal_ take vectorised paths whose last bits depend on the
host CPU's instruction set, so every float here comes from integer draws (torch.randint
on a seeded CPU Generator, an mt19937 stream) and exactly-rounded float32 arithmetic:
identical on the build container and on the GPU box.  This module imports neither the
reference nor the package; the block classes are passed in by each side.

Cases (reference file: the block's definition; the network position it is taken from):
  r18_layer4_0  ResNet-18 layer4.0  BasicBlock(256, 512, stride 2, 1x1 downsample)
                models/resnet.py:22 / :260 (resnet18), input plane 8x8 (224-res: 14x14)
  r18_layer1_0  ResNet-18 layer1.0  BasicBlock(64, 64, stride 1, no downsample): the
                Co <= 64 wave-column alpha backward and the band weight-gradient shapes,
                input plane 16x16 (224-res: 56x56)
  r50_layer1_0  ResNet-50 layer1.0  Bottleneck(64, 64, downsample 64 -> 256)
                models/resnet.py:66, input plane 6x6 (224-res: 56x56)
  mbv2_960      MobileNetV2 features[16]  InvertedResidual(160, 160, 1, expand 6):
                960-channel depthwise conv, models/mobilenetv2.py:24 / :132, plane 7x7
  rgx_g9        RegNetX-3200M stage-3 first block  ResBottleneckBlock(192, 432, stride 2,
                group width 48 -> 9 groups, 1x1 projection), models/regnet.py:113 / :370,
                input plane 10x10
"""
import hashlib

import numpy as np
import torch
import torch.nn as nn

CASES = {
    "r18_layer4_0": ("basic", 256, 512, 8),
    "r18_layer1_0": ("basic1", 64, 64, 16),
    "r50_layer1_0": ("bottleneck", 64, 256, 6),
    "mbv2_960": ("inverted", 160, 160, 7),
    "rgx_g9": ("resbottleneck", 192, 432, 10),
}
N_CALI = 8
ITERS = 20            # fused shifted-scale loop iterations
BRECQ_ITERS = 10      # BRECQ AdaRound iterations
GRAD_STEPS = (0, 5, ITERS - 1)
LONG_ITERS = 625      # the driver's per-block horizon (ShiftedScaleQuant.py:53-55)
LONG_GRAD_STEPS = (0, 125, 312, 469, 624)   # warm-up, both b schedules, the end
BRECQ_GRAD_STEPS = (0, BRECQ_ITERS - 1)
N_SUB = 8192          # sub-sampled entries of a full-size parameter / gradient
WEIGHT_SEED, INPUT_SEED = 2024, 2025

# sum of 4 uniform 16-bit integers: mean 131070, std sqrt(4 * (65536^2 - 1) / 12)
_XN_MEAN = 131070
_XN_INV_STD = float(np.float32(1.0 / 37837.2268))


def xnormal(g, shape):
    """Approximately N(0, 1) from integer draws: exact on any CPU.  Scaled by a MULTIPLY
    with a float32 constant: torch's CPU division by a scalar takes a reciprocal-multiply in
    its vector body and a true division in the scalar tail, and where the tail falls
    depends on the host's vector width."""
    u = torch.randint(0, 65536, (4,) + tuple(shape), generator=g, dtype=torch.int64)
    s = (u.sum(0) - _XN_MEAN).to(torch.float32)          # exact: |s| < 2^18
    return s * _XN_INV_STD


def seed_sha(net):
    """Hash of every seeded parameter / buffer (before any folding)."""
    h = hashlib.sha256()
    for m in net.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear, nn.BatchNorm2d)):
            for t in list(m.parameters(recurse=False)) + list(m.buffers(recurse=False)):
                if t.is_floating_point():
                    h.update(t.detach().float().contiguous().numpy().tobytes())
    return h.hexdigest()


def xuniform(g, shape):
    """U[0, 1) on a 2^-16 grid: exact on any CPU."""
    return torch.randint(0, 65536, tuple(shape), generator=g, dtype=torch.int64).to(torch.float32) * (2.0 ** -16)


def _pow2(v):
    return float(2.0 ** np.round(np.log2(v)))


def _bn_var(g, c, eps=1e-5):
    """Running variances whose std sqrt(var + eps) is EXACTLY 0.5, 1 or 2 in float32, so
    the BN fold (w * gamma / std, beta - gamma * mean / std: quant/fold_bn.py:14-35) is a
    chain of correctly rounded operations with power-of-two divisors -- the same bits
    whichever vector or scalar path a host's torch build takes."""
    k = torch.randint(-1, 2, (c,), generator=g, dtype=torch.int64).numpy()
    std = np.float32(2.0) ** k.astype(np.float32)
    var = (std * std - np.float32(eps)).astype(np.float32)
    assert np.all(np.sqrt((var + np.float32(eps)).astype(np.float32)) == std)
    return torch.from_numpy(var)


def seed_net(net):
    """Kaiming-scale (fan_out, rounded to a power of two) convs, non-trivial BN statistics
    (exact power-of-two stds), small fc: integer draws in module order (the same order on
    both sides: checked through layout() and seed_sha())."""
    g = torch.Generator().manual_seed(WEIGHT_SEED)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.weight.shape[0] * m.weight.shape[2] * m.weight.shape[3]
                m.weight.copy_(xnormal(g, m.weight.shape) * _pow2(np.sqrt(2.0 / fan_out)))
            elif isinstance(m, nn.BatchNorm2d):
                c = m.num_features
                m.running_mean.copy_(xnormal(g, (c,)) * 0.125)
                m.running_var.copy_(_bn_var(g, c, m.eps))
                m.weight.copy_(xuniform(g, (c,)) + 0.5)
                m.bias.copy_(xnormal(g, (c,)) * 0.125)
            elif isinstance(m, nn.Linear):
                m.weight.copy_(xnormal(g, m.weight.shape) * 0.0625)
                m.bias.copy_(xnormal(g, m.bias.shape) * 0.015625)
    return net.eval()


def layout(net):
    """(type, shape) of every seeded module, in seeding order."""
    out = []
    for m in net.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            out.append(f"{type(m).__name__}{tuple(m.weight.shape)}")
        elif isinstance(m, nn.BatchNorm2d):
            out.append(f"BatchNorm2d({m.num_features})")
    return out


def calib_input(case):
    """The block's calibration input: ReLU(N(0,1)) of [N_CALI, C_in, H, W]."""
    _, cin, _, hw = CASES[case]
    g = torch.Generator().manual_seed(INPUT_SEED)
    return torch.relu(xnormal(g, (N_CALI, cin, hw, hw)))


def wrap(block, cout):
    """block -> global pool -> fc: the block is the network's first module (its calibration
    input is fed directly) and first/last layers are left at the block's bit width."""
    return nn.Sequential(block, nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cout, 10))


def sha(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return hashlib.sha256(a.tobytes()).hexdigest()


def sub_idx(n):
    """Fixed sub-sample of a flattened tensor of n entries (all of them when small)."""
    if n <= N_SUB:
        return np.arange(n, dtype=np.int64)
    return np.sort(np.random.RandomState(n % (2 ** 31)).choice(n, N_SUB, replace=False)).astype(np.int64)


def row_l1(a):
    """Per-output-channel L1 norm (float64) of a [Co, ...] tensor."""
    a = np.asarray(a, dtype=np.float64)
    return np.abs(a.reshape(a.shape[0], -1)).sum(axis=1)

"""ResNet-18 downsample (1x1 stride-2) weight gradients: K17's 1x1 GEMM kernel vs the
im2col + hipBLASLt GEMM form (conv_wgrad_gemm), batch 32; plus repeat bit-identity.
usage: python tools/ds_gemm_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from tools.overlap_probe import graph_ms  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for name, (ci, co, hw) in {"layer2.0.ds": (64, 128, 56), "layer3.0.ds": (128, 256, 28),
                           "layer4.0.ds": (256, 512, 14)}.items():
    x = torch.randn(32, ci, hw, hw, device=dev)
    dy = torch.randn(32, co, hw // 2, hw // 2, device=dev)
    ws = (co, ci, 1, 1)
    a = K.conv_wgrad_gemm(x, dy, ws, 2, 0)
    b = K.conv_wgrad_gemm(x, dy, ws, 2, 0)
    k17 = K.conv_wgrad(x, dy, ws, 2, 0, 1)
    out[name] = {"k17_ms": round(graph_ms(lambda: K.conv_wgrad(x, dy, ws, 2, 0, 1)), 4),
                 "gemm_ms": round(graph_ms(lambda: K.conv_wgrad_gemm(x, dy, ws, 2, 0)), 4),
                 "repeat_bit_identical": bool(torch.equal(a, b)),
                 "max_rel_vs_k17": float(((a - k17).abs().max() / k17.abs().max()).item())}
print(json.dumps(out))

"""MIOpen's deterministic conv forward / input gradient vs the same as one fp32 library GEMM
at the ResNet-18 layer3 / layer4 shapes (batch 32):
  forward  y2[Co, N*P]   = W[Co, C*9] @ colT[C*9, N*P]   (col written by the wgrad operands)
  dgrad    dcol[N*P, C*9] = dy2T[N*P, Co] @ W[Co, C*9]    (+ a col2im gather)
usage: python tools/fwd_gemm_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.overlap_probe import graph_ms  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
dev = torch.device("cuda:0")
SHAPES = {"layer3": (256, 256, 14, 1), "layer3.0_s2": (128, 256, 28, 2), "layer4": (512, 512, 7, 1),
          "layer4.0_s2": (256, 512, 14, 2)}
if "--l12" in sys.argv:    # ResNet-18 layer1 / layer2 / layer2.0's stride-2 conv
    SHAPES = {"layer1": (64, 64, 56, 1), "layer2": (128, 128, 28, 1), "layer2.0_s2": (64, 128, 56, 2)}
out = {}
for name, (ci, co, hw, st) in SHAPES.items():
    x = torch.randn(32, ci, hw, hw, device=dev)
    w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
    y = torch.nn.functional.conv2d(x, w, None, st, 1)
    P = y.shape[2] * y.shape[3]
    NP = 32 * P
    g = torch.randn_like(y)
    w2 = w.reshape(co, ci * 9)
    col = torch.randn(NP, ci * 9, device=dev)
    dy2 = torch.randn(co, NP, device=dev)
    flops = 2.0 * co * ci * 9 * NP
    r = {"miopen_fwd_ms": graph_ms(lambda: torch.nn.functional.conv2d(x, w, None, st, 1)),
         "miopen_dgrad_ms": graph_ms(lambda: torch.ops.aten.convolution_backward(
             g, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, (True, False, False))[0]),
         "gemm_fwd_ms": graph_ms(lambda: w2 @ col.t()),
         "gemm_dgrad_ms": graph_ms(lambda: dy2.t() @ w2)}
    r = {k: round(v, 4) for k, v in r.items()}
    r["gemm_fwd_tf"] = round(flops / r["gemm_fwd_ms"] / 1e9, 1)
    r["gemm_dgrad_tf"] = round(flops / r["gemm_dgrad_ms"] / 1e9, 1)
    out[name] = r
print(json.dumps(out))

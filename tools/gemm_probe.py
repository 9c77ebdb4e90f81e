"""fp32 library GEMM rate (torch.matmul -> hipBLASLt / rocBLAS) at the shapes of a
ResNet-18 3x3 conv weight gradient written as one GEMM, dW[Co, Ci*9] = dy[Co, N*P] @
Xcol[N*P, Ci*9] (batch 32), next to the im2col tensor's size; and whether repeated calls
are bit-identical.  usage: python tools/gemm_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.overlap_probe import graph_ms  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"layer1": (64, 64, 56), "layer2": (128, 128, 28), "layer3": (256, 256, 14),
          "layer4": (512, 512, 7)}
out = {}
for name, (ci, co, hw) in SHAPES.items():
    P = 32 * hw * hw
    a = torch.randn(co, P, device=dev)
    b = torch.randn(P, ci * 9, device=dev)
    bt = b.t().contiguous()      # Xcol stored (Ci*9, N*P): the GEMM reads it transposed
    r1 = a @ b
    r2 = a @ b
    flops = 2.0 * co * P * ci * 9
    ms = graph_ms(lambda: a @ b)
    ms_t = graph_ms(lambda: a @ bt.t())
    out[name] = {"M": co, "N": ci * 9, "K": P, "ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                 "ms_bT": round(ms_t, 4), "tflops_bT": round(flops / ms_t / 1e9, 1),
                 "xcol_mb": round(P * ci * 9 * 4 / 1e6, 1), "repeat_bit_identical": bool(torch.equal(r1, r2))}
print(json.dumps(out))

"""The GEMM forward of the small-plane convs (ResNet-18 layer3 / layer4, batch 32): one GEMM
y2[Co, N*P] = W @ col^T then a permute to NCHW (conv_fwd_gemm), against a strided-batched
GEMM per sample y[n] = W @ col_n^T that writes NCHW directly (no permute copy).
usage: python tools/fwd_gemm_layout_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda:0")
for name, (C, H, Co, st) in {"layer3.0.s2": (128, 28, 256, 2), "layer3.3x3": (256, 14, 256, 1),
                             "layer4.0.s2": (256, 14, 512, 2), "layer4.3x3": (512, 7, 512, 1)}.items():
    x = torch.randn(32, C, H, H, device=dev)
    w = torch.randn(Co, C, 3, 3, device=dev) * 0.02
    oh = (H - 1) // st + 1
    P = oh * oh
    col, _ = K.gemm_operands(x, None, w.shape, st, 1, want_col=True, want_dy2=False)
    w2 = w.reshape(Co, C * 9)

    def permuted():
        y2 = torch.matmul(w2, col.t())
        return y2.view(Co, 32, P).permute(1, 0, 2).contiguous().view(32, Co, oh, oh)

    def batched():
        return torch.matmul(w2, col.view(32, P, C * 9).transpose(1, 2)).view(32, Co, oh, oh)

    a, b = permuted(), batched()
    row = {"permuted_ms": round(graph_time_ms(permuted), 4), "batched_ms": round(graph_time_ms(batched), 4),
           "max_rel_diff": float(((a - b).abs().max() / a.abs().max()).item()),
           "batched_repeat_identical": bool(torch.equal(b, batched()))}
    print(json.dumps({name: row}), flush=True)

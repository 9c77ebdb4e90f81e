"""Input gradient of the small-plane 3x3 convs (ResNet-18 layer3 / layer4 conv2, batch 32):
MIOpen's deterministic backward-data against the library GEMM dcol = dy2^T @ W or its
transpose dcol^T = W^T @ dy2 (the col2im gather after it not included).  usage: python tools/dgrad_gemm_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.deterministic = True
for name, (C, H, Co) in {"layer3.3x3": (256, 14, 256), "layer4.3x3": (512, 7, 512)}.items():
    x = torch.randn(32, C, H, H, device=dev)
    w = torch.randn(Co, C, 3, 3, device=dev) * 0.02
    dy = torch.randn(32, Co, H, H, device=dev)
    dy2 = dy.permute(1, 0, 2, 3).reshape(Co, -1).contiguous()
    w2 = w.reshape(Co, C * 9)

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False,
                                                   [0, 0], 1, (True, False, False))[0]

    def gemm():
        return torch.matmul(dy2.t(), w2)

    def gemm_t():          # dcol^T = W^T @ dy2: [C*9, N*P], the col2im gather reads it along p
        return torch.matmul(w2.t(), dy2)

    print(json.dumps({name: {"miopen_det_ms": round(graph_time_ms(miopen), 4),
                             "gemm_dcol_ms": round(graph_time_ms(gemm), 4),
                             "gemm_dcolT_ms": round(graph_time_ms(gemm_t), 4)}}), flush=True)

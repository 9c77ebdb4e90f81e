"""ResNet-18 convs at validation batch 128, forward only: MIOpen (deterministic solvers, and
benchmark-chosen) against the im2col + library GEMM forward (kernels.conv_fwd_gemm).
usage: python tools/val_conv_probe.py"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = {"stem7x7s2": (3, 224, 64, 7, 2, 3), "l1.3x3": (64, 56, 64, 3, 1, 1),
          "l2.0.3x3s2": (64, 56, 128, 3, 2, 1), "l2.3x3": (128, 28, 128, 3, 1, 1),
          "l3.0.3x3s2": (128, 28, 256, 3, 2, 1), "l3.3x3": (256, 14, 256, 3, 1, 1),
          "l4.0.3x3s2": (256, 14, 512, 3, 2, 1), "l4.3x3": (512, 7, 512, 3, 1, 1)}
for name, (C, H, Co, k, st, pad) in SHAPES.items():
    x = torch.randn(128, C, H, H, device=dev)
    w = torch.randn(Co, C, k, k, device=dev) * 0.05
    row = {}
    for det in (True, False):
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, not det
        row[f"miopen_det{int(det)}_ms"] = round(graph_time_ms(lambda: F.conv2d(x, w, None, st, pad)), 4)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        row["gemm_ms"] = round(graph_time_ms(lambda: K.conv_fwd_gemm(x, w, st, pad)[0]), 4)
    except Exception as e:  # noqa: BLE001 -- operands over 2^31 elements
        row["gemm_ms"] = str(e)[:60]
    print(json.dumps({name: row}), flush=True)

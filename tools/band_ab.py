"""K17 band-kernel time (stage 1 + stage 2, the band form forced) on the ResNet-18 band
shapes (batch 32), HIP-graph replay of ssq_conv_wgrad: the A/B harness for band-kernel
changes.  Point SSQ_LIB at another build of libssq.so to time that one.
    python tools/band_ab.py [tag]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda")
SHAPES = {"r18.l1.3x3": (64, 56, 64, 1), "r18.l2.3x3s2": (64, 56, 128, 2),
          "r18.l2.3x3": (128, 28, 128, 1), "r18.l3.3x3s2": (128, 28, 256, 2)}


row = {"lib": os.environ.get("SSQ_LIB", "in-tree"), "tag": sys.argv[1] if len(sys.argv) > 1 else ""}
K.set_wgrad_form(3)
for name, (C, H, Co, st) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(32, C, H, H, device=dev, generator=g)
    oh = (H + 2 - 3) // st + 1
    dy = torch.randn(32, Co, oh, oh, device=dev, generator=g)
    ws = (Co, C, 3, 3)
    row[name] = round(graph_time_ms(lambda: K.conv_wgrad(x, dy, ws, st, 1, 1)) * 1e3, 1)
K.set_wgrad_form(0)
print(json.dumps(row), flush=True)

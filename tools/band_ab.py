"""K17 band-kernel timing on the ResNet-18 band shapes (batch 32), HIP-graph replay of
ssq_conv_wgrad (stage 1 + stage 2): the A/B harness for band-kernel changes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda")
SHAPES = {"l1.3x3": (64, 56, 64, 1), "l2.3x3": (128, 28, 128, 1), "l2.3x3s2": (64, 56, 128, 2),
          "l3.3x3": (256, 14, 256, 1), "l4.3x3": (512, 7, 512, 1)}
row = {"tag": os.environ.get("SSQ_BAND_DEBUG", "0")}
for name, (C, H, Co, st) in SHAPES.items():
    x = torch.randn(32, C, H, H, device=dev)
    oh = (H - 1) // st + 1
    dy = torch.randn(32, Co, oh, oh, device=dev)
    t = graph_time_ms(lambda: K.conv_wgrad(x, dy, (Co, C, 3, 3), st, 1, 1))
    row[name] = round(t * 1e3, 1)
print(json.dumps(row), flush=True)

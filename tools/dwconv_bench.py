"""Depthwise conv forward / input gradient / weight gradient: MIOpen (fastest and
deterministic solvers) vs K18 / K17, MobileNetV2 shapes at batch 32 (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
F = torch.nn.functional
SHAPES = {"f1.dw32@112": (32, 112, 1), "f2.dw96@112s2": (96, 112, 2), "f3.dw144@56": (144, 56, 1),
          "f4.dw144@56s2": (144, 56, 2), "f7.dw192@28s2": (192, 28, 2), "f11.dw384@14": (384, 14, 1),
          "f17.dw960@7": (960, 7, 1)}


def ev(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 1)


for name, (C, H, st) in SHAPES.items():
    x = torch.randn(32, C, H, H, device=dev)
    w = torch.randn(C, 1, 3, 3, device=dev)
    y = F.conv2d(x, w, None, st, 1, 1, C)
    dy = torch.randn_like(y)
    row = {}
    for det in (False, True):
        torch.backends.cudnn.deterministic = det
        row[f"miopen_det{int(det)}"] = {
            "fwd": ev(lambda: F.conv2d(x, w, None, st, 1, 1, C)),
            "dx": ev(lambda: torch.nn.grad.conv2d_input(x.shape, w, dy, st, 1, 1, C)),
            "dw": ev(lambda: torch.nn.grad.conv2d_weight(x, w.shape, dy, st, 1, 1, C))}
    torch.backends.cudnn.deterministic = False
    row["k18_k17"] = {"fwd": ev(lambda: K.dwconv_fwd(x, w, st, 1)),
                      "dx": ev(lambda: K.dwconv_bwd_data(dy, w, x.shape, st, 1)),
                      "dw": ev(lambda: K.conv_wgrad(x, dy, w.shape, st, 1, C))}
    mb = (x.numel() + y.numel()) * 4 / 1e6
    row["plane_MB"] = round(mb, 1)
    print(json.dumps({name: row}), flush=True)

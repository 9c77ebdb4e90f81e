"""Conv weight-gradient time: MIOpen (fastest solvers), MIOpen deterministic, and K17
(ssq_conv_wgrad), for the reconstruction loops' conv shapes at batch 32 (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
SHAPES = {  # name: (C, H, Co, k, stride, pad, groups)
    "r18.l1.3x3": (64, 56, 64, 3, 1, 1, 1), "r18.l2.3x3s2": (64, 56, 128, 3, 2, 1, 1),
    "r18.l2.1x1s2": (64, 56, 128, 1, 2, 0, 1), "r18.l2.3x3": (128, 28, 128, 3, 1, 1, 1),
    "r18.l3.3x3s2": (128, 28, 256, 3, 2, 1, 1), "r18.l3.1x1s2": (128, 28, 256, 1, 2, 0, 1),
    "r18.l3.3x3": (256, 14, 256, 3, 1, 1, 1), "r18.l4.3x3s2": (256, 14, 512, 3, 2, 1, 1),
    "r18.l4.1x1s2": (256, 14, 512, 1, 2, 0, 1), "r18.l4.3x3": (512, 7, 512, 3, 1, 1, 1),
    "mbv2.dw.3x3": (144, 56, 144, 3, 1, 1, 144), "mbv2.dw.3x3s2": (144, 56, 144, 3, 2, 1, 144),
    "rgx.g2.3x3": (96, 56, 96, 3, 1, 1, 2),
    "r50.l1.1x1": (64, 56, 256, 1, 1, 0, 1), "r50.l1.1x1b": (256, 56, 64, 1, 1, 0, 1)}


def ev_time(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


res = {}
for name, (C, H, Co, k, st, pad, g) in SHAPES.items():
    x = torch.randn(32, C, H, H, device=dev)
    w = torch.randn(Co, C // g, k, k, device=dev)
    dy = torch.randn(torch.nn.functional.conv2d(x, w, None, st, pad, 1, g).shape, device=dev)
    row = {}
    for det in (False, True):
        torch.backends.cudnn.deterministic = det
        row[f"miopen_det{int(det)}_us"] = round(ev_time(
            lambda: torch.nn.grad.conv2d_weight(x, w.shape, dy, st, pad, 1, g)), 1)
    torch.backends.cudnn.deterministic = False
    K.set_wgrad_form(1)
    if not K.conv_wgrad_supported(x, w, st, pad, 1, g):
        row["k17_us"] = None
        print(json.dumps({name: row}), flush=True)
        continue
    oh = dy.shape[2]
    flops = 2.0 * 32 * Co * (C // g) * k * k * oh * oh
    for form, tag in ((1, "k17"), (2, "i2c"), (3, "band"), (0, "auto")):
        K.set_wgrad_form(form)
        t = ev_time(lambda: K.conv_wgrad(x, dy, w.shape, st, pad, g))
        row[tag + "_us"] = round(t, 1)
        row[tag + "_tflops"] = round(flops / t / 1e6, 1)
    K.set_wgrad_form(0)
    res[name] = row
    print(json.dumps({name: row}), flush=True)

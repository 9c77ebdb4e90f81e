"""Conv weight-gradient cost under MIOpen's solver settings (deterministic / benchmark),
for the ResNet-18 conv shapes the recon loops differentiate (batch 32)."""
import json
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda")
SHAPES = {  # name: (Ci, H, Co, stride, k)
    "l1_3x3": (64, 56, 64, 1, 3), "l2_3x3s2": (64, 56, 128, 2, 3), "l2_1x1s2": (64, 56, 128, 2, 1),
    "l2_3x3": (128, 28, 128, 1, 3), "l4_3x3": (512, 7, 512, 1, 3)}


def t_wgrad(Ci, H, Co, s, k):
    x = torch.randn(32, Ci, H, H, device=dev)
    w = torch.randn(Co, Ci, k, k, device=dev, requires_grad=True)
    y = F.conv2d(x, w, stride=s, padding=k // 2)
    g = torch.randn_like(y)

    def once():
        return torch.autograd.grad(F.conv2d(x, w, stride=s, padding=k // 2), w, g)[0]
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        once()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 20 * 1e6


res = {}
for det in (False, True):
    for bench in (False, True):
        torch.backends.cudnn.deterministic = det
        torch.backends.cudnn.benchmark = bench
        for name, sh in SHAPES.items():
            res[f"{name} det={int(det)} bench={int(bench)}"] = round(t_wgrad(*sh), 1)
        print(json.dumps(res), flush=True)

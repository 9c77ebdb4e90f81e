"""ResNet-18 downsample (1x1 stride-2) forward: MIOpen (deterministic and benchmark
solvers; it transposes NCHW <-> CNHW around a GEMM) against a strided-batched library GEMM
on the subsampled input (y[n] = W @ x[n, :, ::2, ::2], no transposes), batch 32 (recon) and
128 (validation); plus the GEMM form's error vs the fp64 conv and repeat bit-identity.
usage: python tools/ds_fwd_probe.py"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import graph_time_ms as graph_ms  # noqa: E402

dev = torch.device("cuda:0")


def gemm_fwd(x, w, st):
    xs = x[:, :, ::st, ::st]
    n, c, oh, ow = xs.shape
    y = torch.matmul(w.view(w.shape[0], c), xs.reshape(n, c, oh * ow))
    return y.view(n, w.shape[0], oh, ow)


out = {}
for nb in (32, 128):
    for name, (ci, co, hw) in {"layer2.0.ds": (64, 128, 56), "layer3.0.ds": (128, 256, 28),
                               "layer4.0.ds": (256, 512, 14)}.items():
        x = torch.randn(nb, ci, hw, hw, device=dev)
        w = torch.randn(co, ci, 1, 1, device=dev) * 0.05
        row = {}
        for det in (True, False):
            torch.backends.cudnn.deterministic = det
            torch.backends.cudnn.benchmark = not det
            row[f"miopen_det{int(det)}_ms"] = round(graph_ms(lambda: F.conv2d(x, w, None, 2)), 4)
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
        row["gemm_ms"] = round(graph_ms(lambda: gemm_fwd(x, w, 2)), 4)
        a, b = gemm_fwd(x, w, 2), gemm_fwd(x, w, 2)
        ref = F.conv2d(x.double().cpu(), w.double().cpu(), None, 2)
        mag = F.conv2d(x.double().abs().cpu(), w.double().abs().cpu(), None, 2)
        row["repeat_bit_identical"] = bool(torch.equal(a, b))
        row["max_err_over_mag"] = float(((a.double().cpu() - ref).abs() / mag.clamp_min(1e-30)).max())
        out[f"{name}.b{nb}"] = row
        print(json.dumps({f"{name}.b{nb}": row}), flush=True)

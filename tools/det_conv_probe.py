"""Which convolutions of ResNet-50 / MobileNetV2 / RegNetX-3200M does MIOpen run slowly under
the reference's cudnn.deterministic?  Every distinct conv (input shape at 224x224, weight,
stride, padding, groups) of each network, forward at batch 32: torch's F.conv2d with
deterministic solvers, and K.conv2d (the product path:
depthwise on K18, 1x1 stride-2 as one batched GEMM), each timed as 10 calls in one HIP graph.

    python tools/det_conv_probe.py [archs...]  -> one JSON line per conv, slowest first"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from shiftedscalequantization_amd import kernels as K, nets  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402


def conv_shapes(arch):
    net = nets.ARCHS[arch]().eval()
    seen = {}

    def hook(m, args, out):
        x = args[0]
        key = (tuple(x.shape[1:]), tuple(m.weight.shape), m.stride[0], m.padding[0], m.groups)
        seen.setdefault(key, 0)
        seen[key] += 1

    hs = [m.register_forward_hook(hook) for m in net.modules() if isinstance(m, nn.Conv2d)]
    with torch.no_grad():
        net(torch.zeros(1, 3, 224, 224))
    for h in hs:
        h.remove()
    return seen


def main():
    archs = sys.argv[1:] or ["resnet50", "mobilenetv2", "regnetx_3200m"]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    rows = []
    for arch in archs:
        for (xs, ws, st, pad, groups), count in conv_shapes(arch).items():
            x = torch.empty((32,) + xs, device=dev).normal_(generator=g)
            w = torch.empty(ws, device=dev).normal_(generator=g)
            r = {"arch": arch, "x": xs, "w": ws, "stride": st, "pad": pad, "groups": groups,
                 "count": count}
            torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
            r["torch_det_us"] = round(1e3 * graph_time_ms(
                lambda: torch.nn.functional.conv2d(x, w, None, st, pad, 1, groups), reps=10), 1)
            oh = (xs[1] + 2 * pad - ws[2]) // st + 1
            flop = 2.0 * 32 * ws[0] * ws[1] * ws[2] * ws[3] * oh * oh
            r["torch_det_tflops"] = round(flop / (r["torch_det_us"] * 1e-6) / 1e12, 2)
            with torch.no_grad():
                r["k_conv2d_det_us"] = round(1e3 * graph_time_ms(
                    lambda: K.conv2d(x, w, st, pad, 1, groups), reps=10), 1)
            rows.append(r)
            del x, w
    rows.sort(key=lambda r: -r["torch_det_us"] * r["count"])
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

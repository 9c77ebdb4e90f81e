"""1x1 stride-1 convolutions at batch 32 on every such shape of ResNet-50 / MobileNetV2 /
RegNetX-3200M at 224x224: forward, input gradient and weight gradient on MIOpen under the
reference's cudnn.deterministic (F.conv2d / aten.convolution_backward) against the same
products as one strided-batched library GEMM (y[n] = W @ x[n], dx[n] = W^T @ dy[n];
dW = sum_n dy[n] x[n]^T, K.conv_wgrad_1x1_bmm; K17's 1x1 kernel and the im2col GEMM too), each timed as 10 calls in one HIP graph, with
the GEMM's error against float64 and whether it is bit-identical run to run.

    python tools/conv1x1_probe.py [archs...]  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402
from tools.det_conv_probe import conv_shapes  # noqa: E402


def main():
    archs = sys.argv[1:] or ["resnet50", "mobilenetv2", "regnetx_3200m"]
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    for arch in archs:
        for (xs, ws, st, pad, groups), count in conv_shapes(arch).items():
            if ws[2] != 1 or ws[3] != 1 or st != 1 or pad != 0 or groups != 1:
                continue
            n = 32
            co, c = ws[0], ws[1]
            x = torch.empty((n,) + xs, device=dev).normal_(generator=g)
            w = torch.empty(ws, device=dev).normal_(generator=g)
            dy = torch.empty((n, co) + xs[1:], device=dev).normal_(generator=g)
            p = xs[1] * xs[2]
            w2 = w.view(co, c)
            forms = {
                "fwd_miopen": lambda: torch.nn.functional.conv2d(x, w),
                "fwd_gemm": lambda: torch.matmul(w2, x.view(n, c, p)),
                "dgrad_miopen": lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                    (True, False, False))[0],
                "dgrad_gemm": lambda: torch.matmul(w2.t(), dy.view(n, co, p)),
                "wgrad_miopen": lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                    (False, True, False))[1],
                "wgrad_bmm": lambda: K.conv_wgrad_1x1_bmm(x, dy, ws),
                "wgrad_k17": lambda: K.conv_wgrad(x, dy, ws, 1, 0, 1),
                "wgrad_gemm": lambda: K.conv_wgrad_gemm(x, dy, ws, 1, 0),
            }
            r = {"arch": arch, "x": xs, "w": ws, "count": count,
                 "gflop": round(2.0 * n * co * c * p / 1e9, 3)}
            for k, fn in forms.items():
                try:
                    a, b = fn(), fn()
                except K.A.SSQError as e:  # a K17 / operands size limit
                    r[k + "_us"] = str(e)[:80]
                    continue
                torch.cuda.synchronize()
                r[k + "_us"] = round(1e3 * graph_time_ms(fn, reps=10), 1)
                if not k.endswith("miopen"):
                    r[k + "_identical"] = bool(torch.equal(a, b))
            ref_f = torch.matmul(w2.double(), x.view(n, c, p).double())
            ref_d = torch.matmul(w2.double().t(), dy.view(n, co, p).double())
            r["fwd_gemm_rel"] = ((forms["fwd_gemm"]().double() - ref_f).abs().max()
                                 / ref_f.abs().max()).item()
            r["dgrad_gemm_rel"] = ((forms["dgrad_gemm"]().double() - ref_d).abs().max()
                                   / ref_d.abs().max()).item()
            print(json.dumps(r), flush=True)
            del x, w, dy


if __name__ == "__main__":
    main()

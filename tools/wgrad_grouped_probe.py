"""Grouped 3x3 convolution weight gradients at batch 32 (RegNetX-3200M's 'b' convs, group width
48): K17's implicit-GEMM kernel (ssq_conv_wgrad) against the im2col operands of every channel
(ssq_wgrad_gemm_operands) and ONE strided-batched library GEMM over the groups, each timed as
20 calls in one HIP graph (median of 5 replays), with its error against a float64 reference
and whether it is bit-identical run to run.

    python tools/wgrad_grouped_probe.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (name, N, C, H, stride, groups): RegNetX-3200M stages at 224x224
    ("rgx_s1_b1", 32, 96, 112, 2, 2), ("rgx_s1_b2", 32, 96, 56, 1, 2),
    ("rgx_s2_b1", 32, 192, 56, 2, 4), ("rgx_s2_b2", 32, 192, 28, 1, 4),
    ("rgx_s3_b1", 32, 432, 28, 2, 9), ("rgx_s3_b2", 32, 432, 14, 1, 9),
    ("rgx_s4_b1", 32, 1008, 14, 2, 21), ("rgx_s4_b2", 32, 1008, 7, 1, 21),
]


def grouped_gemm(x, dy, w_shape, st, pad, groups):
    co, cig, r, s = w_shape
    col, dy2 = K.gemm_operands(x, dy, (co, cig * groups, r, s), st, pad)
    np_ = col.shape[0]
    a = dy2.view(groups, co // groups, np_)
    b = col.view(np_, groups, cig * r * s).transpose(0, 1)
    return torch.matmul(a, b).reshape(w_shape)


def main():
    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    for name, n, c, h, st, groups in SHAPES:
        w_shape = (c, c // groups, 3, 3)
        x = torch.empty(n, c, h, h, device=dev).normal_(generator=g).relu_()
        oh = (h + 2 - 3) // st + 1
        dy = torch.empty(n, c, oh, oh, device=dev).normal_(generator=g)
        ref = torch.nn.grad.conv2d_weight(x.double().cpu(), w_shape, dy.double().cpu(), st, 1,
                                          groups=groups)
        out = {"shape": name, "N": n, "C": c, "H": h, "stride": st, "groups": groups,
               "gflop": round(2.0 * n * c * (c // groups) * 9 * oh * oh / 1e9, 3)}
        forms = {"k17": lambda: K.conv_wgrad(x, dy, w_shape, st, 1, groups),
                 "grouped_gemm": lambda: grouped_gemm(x, dy, w_shape, st, 1, groups)}
        for k, fn in forms.items():
            try:
                a, b = fn(), fn()
            except K.A.SSQError as e:          # e.g. K17's LDS tile on 112-wide rows
                out[k] = {"unsupported": str(e)[:120]}
                continue
            torch.cuda.synchronize()
            ms = graph_time_ms(fn, reps=20, rounds=5)
            err = ((a.double().cpu() - ref).abs().max() / ref.abs().max()).item()
            out[k] = {"us": round(ms * 1e3, 2), "tflops": round(out["gflop"] / ms, 1),
                      "rel_err_vs_f64": err, "run_to_run_identical": bool(torch.equal(a, b))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""1x1 convolution weight gradients at batch 32 (the BRECQ / fused loops of configs 3 and 5):
K17's 1x1 kernel (ssq_conv_wgrad) against library-GEMM forms, each timed as 20 calls in one
HIP graph (median of 5 replays), with its error against a float64 reference and whether it is
bit-identical run to run.

    python tools/wgrad1x1_probe.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (name, N, Ci, H, W, Co, stride)
    ("r50_l1_conv1", 32, 64, 56, 56, 64, 1),
    ("r50_l1_conv3", 32, 64, 56, 56, 256, 1),
    ("r50_l1_ds", 32, 64, 56, 56, 256, 1),
    ("rgx_s3b1_a", 32, 192, 28, 28, 432, 1),
    ("rgx_s3b1_c", 32, 432, 14, 14, 432, 1),
    ("rgx_s3b1_proj_s2", 32, 192, 28, 28, 432, 2),
]


def bmm_sum(x, dy, st):
    """sum_n dy[n] @ x[n]^T: one strided-batched GEMM, then the batch summed in order."""
    xs = x[:, :, ::st, ::st] if st > 1 else x
    n, c = xs.shape[:2]
    co = dy.shape[1]
    p = dy.shape[2] * dy.shape[3]
    return torch.matmul(dy.reshape(n, co, p), xs.reshape(n, c, p).transpose(1, 2)).sum(0)


def one_gemm(x, dy, st):
    """dy as [Co, N*P] and x as [N*P, Ci] (CNHW copies), one GEMM."""
    xs = x[:, :, ::st, ::st] if st > 1 else x
    n, c = xs.shape[:2]
    co = dy.shape[1]
    p = dy.shape[2] * dy.shape[3]
    d2 = dy.reshape(n, co, p).transpose(0, 1).reshape(co, n * p)
    x2 = xs.reshape(n, c, p).transpose(1, 2).reshape(n * p, c)
    return torch.matmul(d2, x2)


def main():
    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    for name, n, ci, h, w, co, st in SHAPES:
        x = torch.empty(n, ci, h, w, device=dev).normal_(generator=g).relu_()
        oh, ow = (h - 1) // st + 1, (w - 1) // st + 1
        dy = torch.empty(n, co, oh, ow, device=dev).normal_(generator=g)
        ref = bmm_sum(x.double(), dy.double(), st)
        out = {"shape": name, "N": n, "Ci": ci, "HW": [h, w], "Co": co, "stride": st,
               "gflop": round(2.0 * n * co * ci * oh * ow / 1e9, 3)}
        forms = {"k17": lambda: K.conv_wgrad(x, dy, (co, ci, 1, 1), st, 0, 1).view(co, ci),
                 "bmm_sum": lambda: bmm_sum(x, dy, st),
                 "one_gemm": lambda: one_gemm(x, dy, st)}
        for k, fn in forms.items():
            a, b = fn(), fn()
            torch.cuda.synchronize()
            ms = graph_time_ms(fn, reps=20, rounds=5)
            err = ((a.double() - ref).abs().max() / ref.abs().max()).item()
            out[k] = {"us": round(ms * 1e3, 2), "tflops": round(out["gflop"] / ms, 1),
                      "rel_err_vs_f64": err, "run_to_run_identical": bool(torch.equal(a, b))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

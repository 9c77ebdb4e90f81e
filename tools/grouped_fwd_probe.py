"""The grouped forward GEMM of conv_fwd_grouped_gemm (RegNetX-3200M s3.b1 'b': g = 9, 48
channels per group, stride 2, batch 32) in two orientations over the same im2col matrix,
each with its permute to NCHW, timed as 20 calls in one HIP graph:
  wcol: Y[g] = W[g] @ col[:, g]^T   (G x Cog x NP), then (N, G, Cog, P)
  colw: Y[g] = col[:, g] @ W[g]^T   (G x NP x Cog), then (N, G, Cog, P)

    python tools/grouped_fwd_probe.py  -> one JSON line"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, c, h, g, st = 32, 432, 28, 9, 2
    x = torch.randn(n, c, h, h, device=dev)
    w = torch.randn(c, c // g, 3, 3, device=dev)
    k = (c // g) * 9
    col, _ = K.gemm_operands(x, None, (c, c, 3, 3), st, 1, want_col=True, want_dy2=False)
    oh = (h + 2 - 3) // st + 1
    w3 = w.reshape(g, c // g, k)
    colg = col.view(-1, g, k)

    def wcol():
        y = torch.matmul(w3, colg.permute(1, 2, 0))
        return y.view(g, c // g, n, oh * oh).permute(2, 0, 1, 3).contiguous()

    def colw():
        y = torch.matmul(colg.transpose(0, 1), w3.transpose(1, 2))
        return y.view(g, n, oh * oh, c // g).permute(1, 0, 3, 2).contiguous()

    a, b = wcol(), colw()
    out = {"max_abs_diff": float((a - b).abs().max())}
    for name, fn in (("wcol", wcol), ("colw", colw),
                     ("wcol_gemm_only", lambda: torch.matmul(w3, colg.permute(1, 2, 0))),
                     ("colw_gemm_only", lambda: torch.matmul(colg.transpose(0, 1), w3.transpose(1, 2))),
                     ("miopen", lambda: torch.nn.functional.conv2d(x, w, None, st, 1, 1, g))):
        out[name + "_us"] = round(1e3 * graph_time_ms(fn, reps=20, rounds=5), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

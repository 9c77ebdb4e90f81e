"""1x1 stride-2 weight gradients (the ResNet downsamples) at batch 32: K17's 1x1 kernel, the
im2col GEMM (operands + one GEMM) and one strided-batched GEMM + batch sum on the subsampled
input the forward GEMM already made contiguous (conv1x1_fwd_gemm's xs), each timed as 20
calls in one HIP graph.

    python tools/ds_wgrad_probe.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (name, C, H, Co): ResNet-18 layer2.0 / 3.0 / 4.0, ResNet-50 layer2.0 / 3.0 / 4.0,
    # RegNetX-3200M s2.b1 / s3.b1 / s4.b1
    ("r18_l2", 64, 56, 128), ("r18_l3", 128, 28, 256), ("r18_l4", 256, 14, 512),
    ("r50_l2", 256, 56, 512), ("r50_l3", 512, 28, 1024), ("r50_l4", 1024, 14, 2048),
    ("rgx_s2", 96, 56, 192), ("rgx_s3", 192, 28, 432), ("rgx_s4", 432, 14, 1008)]


def main():
    dev = torch.device("cuda", 0)
    for name, c, h, co in SHAPES:
        x = torch.randn(32, c, h, h, device=dev)
        oh = h // 2
        dy = torch.randn(32, co, oh, oh, device=dev)
        ws = (co, c, 1, 1)
        xs = x[:, :, ::2, ::2].contiguous()
        ref = K.conv_wgrad(x, dy, ws, 2, 0, 1)
        r = {"shape": name}
        forms = {"k17": lambda: K.conv_wgrad(x, dy, ws, 2, 0, 1),
                 "im2col_gemm": lambda: K.conv_wgrad_gemm(x, dy, ws, 2, 0),
                 "bmm_on_xs": lambda: K.conv_wgrad_1x1_bmm(xs, dy, ws)}
        for k, fn in forms.items():
            try:
                out = fn()
            except K.A.SSQError as e:
                r[k] = str(e)[:60]
                continue
            r[k + "_us"] = round(1e3 * graph_time_ms(fn, reps=20, rounds=5), 1)
            r[k + "_rel"] = float((out - ref).abs().max() / ref.abs().max())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

"""ssq_wgrad_gemm_operands' im2col matrix (col only) at batch 32 on the shapes the recon loops
build it for -- ResNet-18 layer3 / layer4 3x3 convs (stride 1 and 2), RegNetX-3200M s3.b1's
g = 9 'b' conv -- each as 20 calls in one HIP graph, with the bytes it writes.

    python tools/operands_probe.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (name, C, H, Co, stride)
    ("r18_layer3_3x3", 256, 14, 256, 1), ("r18_layer3.0_s2", 128, 28, 256, 2),
    ("r18_layer4_3x3", 512, 7, 512, 1), ("r18_layer4.0_s2", 256, 14, 512, 2),
    ("rgx_s3.b1_g9_s2", 432, 28, 432, 2)]


def main():
    dev = torch.device("cuda", 0)
    for name, c, h, co, st in SHAPES:
        x = torch.randn(32, c, h, h, device=dev)
        ws = (co, c, 3, 3)
        fn = lambda: K.gemm_operands(x, None, ws, st, 1, want_col=True, want_dy2=False)  # noqa
        col, _ = fn()
        ms = graph_time_ms(fn, reps=20, rounds=5)
        mb = col.numel() * 4 / 1e6
        print(json.dumps({"shape": name, "us": round(ms * 1e3, 2), "col_MB": round(mb, 1),
                          "TB_s": round(mb / ms / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()

"""Depthwise 3x3 weight gradients (K17's wgrad_dw_small / wgrad_dw_stage1) at batch 32 on
every depthwise shape of MobileNetV2 at 224x224, each timed as 20 calls in one HIP graph
(median of 5 replays), with the bytes of x and dy it must read.

    python tools/dw_wgrad_probe.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (C, H, stride): MobileNetV2 features.1 .. features.17
    (32, 112, 1), (96, 112, 2), (144, 56, 1), (144, 56, 2), (192, 28, 1), (192, 28, 2),
    (384, 14, 1), (576, 14, 1), (576, 14, 2), (960, 7, 1)]


def main():
    dev = torch.device("cuda", 0)
    n = 32
    for c, h, st in SHAPES:
        x = torch.randn(n, c, h, h, device=dev)
        oh = (h + 2 - 3) // st + 1
        dy = torch.randn(n, c, oh, oh, device=dev)
        ms = graph_time_ms(lambda: K.conv_wgrad(x, dy, (c, 1, 3, 3), st, 1, c), reps=20, rounds=5)
        mb = (x.numel() + dy.numel()) * 4 / 1e6
        print(json.dumps({"N": n, "C": c, "H": h, "stride": st, "us": round(ms * 1e3, 2),
                          "MB": round(mb, 2), "TB_s": round(mb / ms / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()

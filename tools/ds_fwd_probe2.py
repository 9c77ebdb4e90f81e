"""1x1 stride-2 forwards whose output plane is 100-400 pixels (FWD_1X1_GEMM leaves them to
MIOpen): MIOpen's deterministic forward vs K.conv1x1_fwd_gemm, each as 10 calls in one HIP graph.

    python tools/ds_fwd_probe2.py  -> one JSON line per shape"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

SHAPES = [  # (C, H, Co): RegNetX-3200M s2.b1 / s3.b1 proj, ResNet-50 layer2.0 / layer3.0
    (96, 56, 192), (192, 28, 432), (256, 56, 512), (512, 28, 1024)]


def main():
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dev = torch.device("cuda", 0)
    for c, h, co in SHAPES:
        x = torch.randn(32, c, h, h, device=dev)
        w = torch.randn(co, c, 1, 1, device=dev)
        r = {"C": c, "H": h, "Co": co}
        r["miopen_us"] = round(1e3 * graph_time_ms(
            lambda: torch.nn.functional.conv2d(x, w, None, 2), reps=10), 1)
        r["gemm_us"] = round(1e3 * graph_time_ms(lambda: K.conv1x1_fwd_gemm(x, w, 2), reps=10), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

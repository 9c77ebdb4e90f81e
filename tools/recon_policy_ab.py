"""Recon iters/s per ResNet-18 block under each conv weight-gradient policy
(kernels.WGRAD_POLICY: MIOpen's choice vs K17 ssq_conv_wgrad), cudnn.deterministic off/on."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import run_block  # noqa: E402

dev = torch.device("cuda")
blocks = sys.argv[1].split(",") if len(sys.argv) > 1 else ["layer1.0", "layer2.0", "layer3.0",
                                                           "layer4.0"]
for det in (False, True):
    torch.backends.cudnn.deterministic = det
    for pol in ("never", "always"):
        K.WGRAD_POLICY = pol
        row = {b: round(run_block(dev, b, iters=100, warmup=10), 1) for b in blocks}
        print(json.dumps({"deterministic": det, "policy": pol, "iters_per_s": row}), flush=True)

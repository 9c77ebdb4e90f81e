"""Fused shifted-scale recon iteration rate on ResNet-18 blocks under the e2e settings:
bias_cal (gamma^z/phi^z learned) and MIOpen deterministic solvers, each on/off."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import run_block  # noqa: E402

dev = torch.device("cuda")
res = {}
for det in (False, True):
    torch.backends.cudnn.deterministic = det
    for bias_cal in (False, True):
        for blk in ("layer1.0", "layer2.0"):
            run_block(dev, blk, iters=20, warmup=5, bias_cal=bias_cal)      # solver setup
            r = run_block(dev, blk, iters=200, warmup=20, bias_cal=bias_cal)
            res[f"{blk} det={int(det)} bias_cal={int(bias_cal)}"] = round(r, 1)
            print(json.dumps({k: v for k, v in res.items()}), flush=True)

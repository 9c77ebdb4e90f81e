"""Deterministic-solver fused recon loop on chosen ResNet-18 blocks (bench.py's recon
workload): iters/s per block.  For A/B runs of an env knob, and under rocprofv3
--kernel-trace for per-kernel durations (tools/trace_avg.py --groups=<n blocks>).
    python tools/recon_blocks.py [iters] [block ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import run_block  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
blocks = sys.argv[2:] or ["layer3.1", "layer4.1"]
torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
out = {}
for b in blocks:
    out[b] = round(run_block(torch.device("cuda"), b, iters=iters, warmup=20)["ips"], 1)
print(json.dumps(out), flush=True)

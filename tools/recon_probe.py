"""Why does layer4.0 recon slow down inside bench.py?  Layer4.0 iters/s fresh, after the
bench's q/dq workload, and with cudnn.benchmark (MIOpen find) on."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.recon_bench import run_block  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda")
mode = sys.argv[1]
if mode == "bench_first":
    act, d_a, z_a, weights, dws, zws, bits = bench.make_workload(dev, 0, 1024)
    y = torch.empty_like(act)
    from shiftedscalequantization_amd import kernels as K
    for _ in range(20):
        K.fake_quant_fwd(act, d_a, z_a, 4)
        K.fake_quant_multi(weights, dws, zws, bits)
    big = torch.empty(8192, 2048, 3, 3, device=dev).normal_(0.0, 0.02)
    del big
if mode == "benchmark":
    torch.backends.cudnn.benchmark = True
for b in ("layer1.0", "layer4.0"):
    print(json.dumps({"mode": mode, b: round(run_block(dev, b, iters=100, warmup=10), 1)}), flush=True)

"""Device time of the reconstruction loss pass (K11, value + gradient, target rows read in
place) and of the fused epilogue backward at the ResNet-18 block-output shapes (batch 32):
HIP-graph replay, median of 5.  Run twice with SSQ_LOSS_ONE_LAUNCH=0/1 for the A/B of the
loss value's finalisation."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402
from shiftedscalequantization_amd.recon_bench import graph_time_ms  # noqa: E402

dev = torch.device("cuda")
for C, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
    pred = torch.randn(32, C, H, H, device=dev).relu_()
    cache = torch.randn(1024, C, H, H, device=dev)
    idx = torch.randperm(1024, device=dev)[:32]
    t = graph_time_ms(lambda: K.lp_loss_and_grad(pred, K.Rows(cache, idx), 2.0, relu_mask=True))
    n = pred.numel()
    print(json.dumps({"shape": [32, C, H, H], "loss_us": round(t * 1e3, 2),
                      "loss_gbs": round(12 * n / t / 1e6, 1),
                      "one_launch": os.environ.get("SSQ_LOSS_ONE_LAUNCH", "0")}), flush=True)

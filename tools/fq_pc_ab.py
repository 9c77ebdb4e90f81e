"""Per-channel W2 q/dq of the [8192,2048,3,3] weight (bench.py's roofline_per_channel):
HIP-event time on the launch stream, GB/s at 8 B/elem."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shiftedscalequantization_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
big = torch.empty(8192, 2048, 3, 3, device=dev).normal_(0.0, 0.02)
d, z, _ = K.scale_init(big, 2, False, True, "max")
y = torch.empty_like(big)
ms = bench.time_events(lambda: K.fake_quant_fwd(big, d, z, 2, out=y), 10, dev)
print(json.dumps({"ms": round(ms, 4),
                  "gbs": round(8.0 * big.numel() / (ms * 1e-3) / 1e9, 1)}), flush=True)

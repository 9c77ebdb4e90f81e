"""Run K17 (ssq_conv_wgrad) on one conv shape a few times: the target of rocprofv3 PMC
passes.  usage: python tools/wgrad_one.py C H Co k stride pad groups [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd import kernels as K  # noqa: E402

C, H, Co, k, st, pad, g = (int(v) for v in sys.argv[1:8])
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 10
dev = torch.device("cuda")
x = torch.randn(32, C, H, H, device=dev)
w_shape = (Co, C // g, k, k)
oh = (H + 2 * pad - k) // st + 1
dy = torch.randn(32, Co, oh, oh, device=dev)
for _ in range(reps):
    K.conv_wgrad(x, dy, w_shape, st, pad, g)
torch.cuda.synchronize()
print("done")

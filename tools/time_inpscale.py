"""Time the ChannelQuantMSE input-scale search (K10) on a 512x256x3x3 W2 layer at
level 1024 (the reference's largest setting)."""
import time

import torch

from shiftedscalequantization_amd import kernels as K

w = torch.randn(512, 256, 3, 3, device="cuda") * 0.05
d, z, r = K.scale_init(w, 2, False, True, "max")
K.inpscale_search(w, d, r, 2, 1024, 2.0)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    K.inpscale_search(w, d, r, 2, 1024, 2.0)
torch.cuda.synchronize()
print("inpscale_search 512x256x3x3 level 1024: %.3f ms" % ((time.perf_counter() - t) / 10 * 1e3))
